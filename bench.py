#!/usr/bin/env python3
"""Benchmark: env-steps/s of the fused Skillshot step kernel on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs 65536]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json metric "env-steps/sec (whole node) at 65536 self-play
envs"): every GPU steps 65,536 games (weak scaling:
envs shard by global id, no data-path collective) with the random policy.
One bench step = one k_step launch over all of a GPU's games: both players'
do_actions (SkillshotLearner.py:206-213) + game_tick (SkillshotGame.py:115-122)
+ done + random auto-reset.  Actions are Philox uniform(-1,1) float32
pre-generated into HBM (K4, not timed), a distinct 1 MiB slab per tick, read
from a ring larger than the 256 MiB Infinity Cache.  The K timed steps are
replayed from hipGraphs of `--graph-len` captured launches (the engine's RNG
step counter lives on device, so replays stay correctly keyed).

Roofline: algorithmic bytes per env-step = 193 B (state 88 B read + 88 B
written, actions 16 B, done 1 B: SURVEY.md §8(d)); average launch duration =
HIP-event span of the timed region on the launch stream / K.  cpu_baseline: the C oracle (a port of the
reference step) on one host core over a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (whole node) at 65536 self-play envs; 1/2/4/8 GPU scaling"
BYTES_PER_ENV_STEP = 193  # SURVEY.md §8(d) step-only contract
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=4000)
    p.add_argument("--warmup", type=int, default=400)
    p.add_argument("--envs", type=int, default=65536, help="games per GPU")
    p.add_argument("--tick-limit", type=int, default=2000)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--graph-len", type=int, default=400, help="launches per captured hipGraph")
    p.add_argument("--action-ring", type=int, default=400, help="distinct per-tick action slabs in HBM")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--cpu-cores", type=int, default=16, help="host cores for the CPU baseline (the box's share)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-rollout", action="store_true")
    p.add_argument("--no-large", action="store_true", help="skip the 4 M-game HBM-bound secondary measurement")
    p.add_argument("--no-strong", action="store_true", help="skip the fixed-65,536-total secondary measurement")
    p.add_argument("--no-learner", action="store_true", help="skip the DDPG-in-the-loop secondary measurement (N=1)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_k_step.json"))
    return p.parse_args()


def cpu_baseline(n_envs, seconds, tick_limit, seed, cores):
    """C oracle (port of the reference step, oracle/skillshot_oracle.c): the
    same workload (random policy, fused step, auto-reset) on `cores` host
    cores, one process per core on its own slice of the games
    (oracle/cpu_bench.py), each bounded to about `seconds` of CPU work; the
    one-core rate is measured first on the full batch."""
    import subprocess
    root = os.path.dirname(os.path.abspath(__file__))
    from oracle import cpu_bench
    one = cpu_bench.run(n_envs, seconds / 2, seed=seed, tick_limit=tick_limit)
    per = n_envs // cores
    procs = [subprocess.Popen([sys.executable, "-m", "oracle.cpu_bench", "--envs", str(per), "--env-offset",
                               str(c * per), "--seconds", str(seconds), "--seed", str(seed), "--tick-limit",
                               str(tick_limit)], cwd=root, stdout=subprocess.PIPE, text=True)
             for c in range(cores)]
    outs = [json.loads(p.communicate()[0].strip().splitlines()[-1]) for p in procs]
    rate = sum(o["env_steps_per_s"] for o in outs)
    # the pure-Python restatement on config 1 (one game, one core), and the
    # reference-equivalent rate through the ratio measured where the
    # reference is importable (tools/ref_ratio.py -> profiles/ref_vs_pyoracle.json)
    py = cpu_bench.run_python(min(5.0, seconds / 2), seed=seed, tick_limit=tick_limit)["env_steps_per_s"]
    ratio_path = os.path.join(root, "profiles", "ref_vs_pyoracle.json")
    ratio = json.load(open(ratio_path)) if os.path.exists(ratio_path) else None
    python_leg = dict(pyoracle_env_steps_per_s_1core=py, procedure="SURVEY 8(d) config 1 (game_tick + actions)")
    if ratio:
        python_leg.update(ratio_pyoracle_over_reference=ratio["ratio_pyoracle_over_reference"],
                          reference_equivalent_env_steps_per_s_1core=py / ratio["ratio_pyoracle_over_reference"],
                          ratio_source="profiles/ref_vs_pyoracle.json")
    return dict(value=rate, unit="env-steps/s", cores=cores, kind="port", python_restatement=python_leg,
                sample=f"C oracle (oracle/skillshot_oracle.c, restatement of the reference step): {cores} processes "
                       f"x {per} games for {seconds:.0f} s each ({sum(o['ticks'] for o in outs) // cores} ticks "
                       f"per process on average); one core on all {n_envs} games: "
                       f"{one['env_steps_per_s']:.4g} env-steps/s; reference Python on the survey host: "
                       f"59.2k env-steps/s per core (BASELINE.md)")


def large_batch_rate(dev, args, rank, n=1 << 22, launches=60, ring=8):
    """k_step at n games per GPU, graph-replayed, HIP-event timed (HBM-bound
    regime: 193 B x n per launch)."""
    import ctypes
    from skillshot_learning_amd import VecSkillshotGame
    env = VecSkillshotGame(n, device=dev, seed=args.seed + 1, env_offset=rank * n, tick_limit=args.tick_limit,
                           random_positions=True)
    st = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(st):
        env.reset(random_positions=True)
        acts = env.gen_random_actions(ring)
        done = torch.empty(n, dtype=torch.uint8, device=dev)
    st.synchronize()
    slab, sp = 16 * n, ctypes.c_void_p(st.cuda_stream)

    def launch(t):
        env.step_raw(ctypes.c_void_p(acts.data_ptr() + (t % ring) * slab), ctypes.c_void_p(done.data_ptr()), stream=sp)

    with torch.cuda.stream(st):
        for t in range(2):
            launch(t)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        for t in range(launches):
            launch(t)
    with torch.cuda.stream(st):
        g.replay()
    st.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        e0.record()
        g.replay()
        e1.record()
    st.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / launches
    gbs = BYTES_PER_ENV_STEP * n / (us * 1e-6) / 1e9
    env.close()
    del acts, done
    return dict(envs_per_gpu=n, kernel="k_step (auto variant)", us_per_launch=us, env_steps_per_s_per_gpu=n / (us * 1e-6),
                achieved_gbs=gbs, frac=gbs / HBM_PEAK_GBS,
                note="state 369 MB > Infinity Cache: the HBM-bound regime; reported beside, not as, the headline")


def strong_scaling_rate(dev, args, rank, world, total=65536, launches=2000, G=400):
    """BASELINE config-5 reading of the metric: 65,536 games in total split
    over the ranks (65,536 / world per GPU), same fused tick; aggregate
    env-steps/s over max-over-ranks wall time (barriers around)."""
    import ctypes
    from skillshot_learning_amd import VecSkillshotGame
    n = total // world
    env = VecSkillshotGame(n, device=dev, seed=args.seed + 2, env_offset=rank * n, tick_limit=args.tick_limit,
                           random_positions=True)
    st = torch.cuda.Stream(device=dev)
    ring = G
    with torch.cuda.stream(st):
        env.reset(random_positions=True)
        acts = env.gen_random_actions(ring)
        done = torch.empty(n, dtype=torch.uint8, device=dev)
    st.synchronize()
    slab, sp = 16 * n, ctypes.c_void_p(st.cuda_stream)

    def launch(t):
        env.step_raw(ctypes.c_void_p(acts.data_ptr() + (t % ring) * slab), ctypes.c_void_p(done.data_ptr()), stream=sp)

    with torch.cuda.stream(st):
        for t in range(2):
            launch(t)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        for t in range(G):
            launch(t)
    with torch.cuda.stream(st):
        g.replay()
    st.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(st):
        for _ in range(launches // G):
            g.replay()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    steps = (launches // G) * G
    env.close()
    return dict(total_envs=total, envs_per_gpu=n, n_gpus=world, env_steps_per_s=total * steps / el,
                us_per_tick=el * 1e6 / steps, scaling="strong",
                note="fixed 65,536 games over all GPUs (launch-bound per GPU at 8,192); reported beside the "
                     "weak-scaling headline")


def learner_rate(envs, ticks=200, batch=4096):
    """Configs 3 / 5 on one GPU: per tick the parameter-noise
    actor forward for both players of every game, the fused env step with
    obs/reward/auto-reset, 2N transitions into the HBM replay ring, one critic
    + actor update (fused MFMA kernels, in-kernel bootstrap target) on a
    `batch` sample, soft target update and actor repack — replayed as one
    captured hipGraph per 2 ticks (SkillshotLearner.tick_graph)."""
    from skillshot_learning_amd.learner import SkillshotLearner
    L = SkillshotLearner(n_envs=envs, seed=0, exploration="param_noise", tick_limit=2000,
                         replay_capacity=1 << 20, gamma=0.99, tau=0.005)
    tg = L.tick_graph(batch=batch, updates_per_tick=1, ticks_per_graph=2)
    tg.run(10)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(tg.stream)
    tg.run(ticks // 2)
    e1.record(tg.stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    n_ticks = (ticks // 2) * 2
    out = dict(envs_per_gpu=envs, ticks=n_ticks, batch=batch, exploration="param_noise", updates_per_tick=1,
               env_steps_per_s=envs * n_ticks / el, ms_per_tick=el * 1e3 / n_ticks,
               gpu_ms_per_tick=e0.elapsed_time(e1) / n_ticks, episodes=L.game_environment.counters())
    del tg, L
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # one rank per GPU over RCCL; SK_BENCH_BACKEND=gloo rehearses the
        # multi-rank path with several ranks sharing the GPUs there are
        backend = os.environ.get("SK_BENCH_BACKEND", "nccl")
        local = local % max(torch.cuda.device_count(), 1) if backend == "gloo" else local
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from skillshot_learning_amd import VecSkillshotGame

    n = args.envs
    env = VecSkillshotGame(n, device=dev, seed=args.seed, env_offset=rank * n, tick_limit=args.tick_limit,
                           random_positions=True)
    stream = torch.cuda.Stream(device=dev)
    G = max(2, args.graph_len - (args.graph_len % 2))  # even: keeps the step-slot parity invariant
    ring = max(G, args.action_ring)
    with torch.cuda.stream(stream):
        env.reset(random_positions=True)
        actions = env.gen_random_actions(ring)  # [ring, 2, N, 2] f32, 16 B/env/tick
        done = torch.empty(n, dtype=torch.uint8, device=dev)
    stream.synchronize()

    a_ptr0 = actions.data_ptr()
    slab = 2 * n * 2 * 4
    d_ptr = done.data_ptr()
    import ctypes
    sp = ctypes.c_void_p(stream.cuda_stream)

    def launch(t):
        env.step_raw(ctypes.c_void_p(a_ptr0 + (t % ring) * slab), ctypes.c_void_p(d_ptr), stream=sp)

    # capture one graph of G launches (eager warm-up first so code objects load)
    with torch.cuda.stream(stream):
        for t in range(4):
            launch(t)
    stream.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=stream):
        for t in range(G):
            launch(t)
    stream.synchronize()

    def run(k):
        """k launches: whole graph replays, remainder eager (parity-safe)."""
        with torch.cuda.stream(stream):
            for _ in range(k // G):
                graph.replay()
            for t in range(k % G):
                launch(t)

    env.clear_counters()
    run(args.warmup)
    stream.synchronize()

    K = args.steps
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        ev0.record()
    run(K)
    with torch.cuda.stream(stream):
        ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ev_ms = ev0.elapsed_time(ev1)
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    total_env_steps = n * world * K
    value = total_env_steps / elapsed

    # ---- roofline: the timed region is K back-to-back k_step launches on
    # `stream` (graph replays), so the HIP-event span / K is the kernel's
    # average launch duration (rocprofv3 --stats reports the same figure).
    kern_ms = ev_ms / K
    achieved = BYTES_PER_ENV_STEP * n / (kern_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("envs") == n:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    counters = env.counters()

    # ---- secondary: register-resident multi-tick random-policy kernel
    rollout = None
    if not args.no_rollout:
        ticks = 200
        with torch.cuda.stream(stream):
            env.rollout_random(ticks)
        stream.synchronize()
        r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        with torch.cuda.stream(stream):
            r0.record()
            for _ in range(reps):
                env.rollout_random(ticks)
            r1.record()
        stream.synchronize()
        rms = r0.elapsed_time(r1)
        rollout = dict(kernel="k_rollout_random", ticks_per_launch=ticks,
                       env_steps_per_s_per_gpu=n * ticks * reps / (rms * 1e-3),
                       note="state held in registers across ticks; reported beside, not as, the headline")

    # ---- secondary: the same k_step tick at 4 M games per GPU (369 MB of
    # state: past the 256 MB Infinity Cache, so truly HBM-bound, not
    # launch-bound) — SURVEY §7 hard part 3; reported beside the headline
    large = None
    if not args.no_large:
        large = large_batch_rate(dev, args, rank)
    strong = None
    if world > 1 and not args.no_strong:
        strong = strong_scaling_rate(dev, args, rank, world)

    # ---- secondary: the DDPG learner in the loop (configs 3 and 5 on one GPU)
    learner = None
    if world == 1 and not args.no_learner:
        learner = {"config3": learner_rate(4096), "config5_1gpu": learner_rate(65536),
                   "note": "env step + param-noise actor + replay insert/sample + critic/actor update per tick; "
                           "reported beside, not as, the headline"}

    cpu = None
    if world == 1 and not args.no_cpu_baseline:  # N=1 only (the CPU baseline is a per-box figure)
        cpu = cpu_baseline(n, args.cpu_seconds, args.tick_limit, args.seed,
                           max(1, min(args.cpu_cores, os.cpu_count() or 1)))

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / K,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": f"config-2 step kernel: {n} games/GPU, random policy (Philox f32 actions pre-generated "
                            f"in HBM), fused k_step per tick (do_actions x2 + game_tick + done + random "
                            f"auto-reset), tick_limit {args.tick_limit}",
                "envs_per_gpu": n,
                "total_envs": n * world,
                "global_batch": n * world,
                "parallelism": f"env-shard dp{world}",
                "graph_len": G,
                "event_ms_per_step": ev_ms / K,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": "k_step",
                "bytes_per_env_step": BYTES_PER_ENV_STEP,
                "kernel_us": kern_ms * 1e3,
            },
            "cpu_baseline": cpu,
            "episodes": counters,
            "rollout_random": rollout,
            "large_batch": large,
            "learner": learner,
            "strong_scaling": strong if strong is not None else (
                {"total_envs": n, "n_gpus": 1, "env_steps_per_s": value, "scaling": "strong",
                 "note": "N=1: the headline itself"} if world == 1 and n == 65536 else None),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    env.close()


if __name__ == "__main__":
    main()
