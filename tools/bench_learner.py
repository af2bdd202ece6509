"""Learner-in-the-loop throughput.

    python tools/bench_learner.py [--envs 4096] [--ticks 200] [--batch 4096] [--updates 1]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/bench_learner.py ...

Per tick and GPU: param-noise actor forward for both players of every game
(fused MFMA kernel), fused env step with obs/reward/auto-reset, 2N
transitions into the HBM replay ring, `--updates` critic+actor updates on a
`--batch` sample (multi-GPU: grads all-reduced over RCCL, minibatch
all-gathered), actor repack.  Prints one JSON line with env-steps/s and the
per-phase split measured with HIP events.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=4096)
    p.add_argument("--ticks", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("--updates", type=int, default=1)
    p.add_argument("--exploration", default="param_noise")
    p.add_argument("--graph", action="store_true", help="replay the tick as one captured hipGraph (1 GPU)")
    a = p.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from skillshot_learning_amd.learner import STATE_DIM, ACTION_DIM, SkillshotLearner
    L = SkillshotLearner(n_envs=a.envs, seed=0, env_offset=rank * a.envs, exploration=a.exploration,
                         tick_limit=2000, replay_capacity=1 << 20, gamma=0.99, tau=0.005)
    g = L.game_environment
    obs = L.prepare_states()
    phases = ("act", "step", "replay_add", "update")
    ev = {k: [] for k in phases}

    def tick(timed):
        nonlocal obs
        e = [torch.cuda.Event(enable_timing=True) for _ in range(len(phases) + 1)] if timed else None
        if timed:
            e[0].record()
        act = L.model_act(obs)
        if timed:
            e[1].record()
        out = L.do_actions(act, reset_obs=True)
        if timed:
            e[2].record()
        L.replay.add(obs.reshape(-1, STATE_DIM), act.reshape(-1, ACTION_DIM), out["reward"].reshape(-1),
                     out["obs"].reshape(-1, STATE_DIM), out["done"].float().repeat(2))
        obs = out["obs_reset"]
        if timed:
            e[3].record()
        for _ in range(a.updates):
            L.replay_update(a.batch)
        L._refresh_actor_pack()
        if timed:
            e[4].record()
            for k, name in enumerate(phases):
                ev[name].append((e[k], e[k + 1]))

    if a.graph:
        tg = L.tick_graph(batch=a.batch, updates_per_tick=a.updates, ticks_per_graph=2)
        tg.run(max(a.warmup // 2, 1))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream())  # TickGraph.run replays on the caller's stream
        tg.run(a.ticks // 2)
        e1.record(torch.cuda.current_stream())
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        ticks = (a.ticks // 2) * 2
        print(json.dumps(dict(
            metric="env-steps/s with DDPG learner in the loop", value=a.envs * ticks / el, unit="env-steps/s",
            n_gpus=1, envs_per_gpu=a.envs, ticks=ticks, batch_per_rank=a.batch, updates_per_tick=a.updates,
            exploration=a.exploration, mode="hipgraph (2 ticks per replay)", ms_per_tick=el * 1e3 / ticks,
            gpu_ms_per_tick=e0.elapsed_time(e1) / ticks, replay_size=L.replay.size,
            episodes=g.counters())), flush=True)
        return
    for _ in range(max(a.warmup, 2)):
        tick(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.ticks):
        tick(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    split = {k: sum(x.elapsed_time(y) for x, y in v) * 1e3 / len(v) for k, v in ev.items()}
    if rank == 0:
        print(json.dumps(dict(
            metric="env-steps/s with DDPG learner in the loop", value=a.envs * world * a.ticks / el,
            unit="env-steps/s", n_gpus=world, envs_per_gpu=a.envs, ticks=a.ticks, batch_per_rank=a.batch,
            updates_per_tick=a.updates, exploration=a.exploration, ms_per_tick=el * 1e3 / a.ticks,
            us_per_phase=split, episodes=g.counters())), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
