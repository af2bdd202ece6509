"""A/B sweep of step-kernel variants x batch sizes (graph-replayed fused step).

    python tools/sweep.py [--variants 0,1] [--envs 65536,262144,1048576] [--steps 2000]
Prints one JSON line per (variant, N): us/step, env-steps/s, GB/s at 193 B/env-step.
The 'empty' / 'copy' floor variants need a diagnostic build with csrc/sk_diag.hip:
    tools/build_variant.sh ab/diag.so && SK_LIB_PATH=$PWD/ab/diag.so python tools/sweep.py ...
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(variant, n, steps, graph_len, ring, obs=False):
    """variant 0/1 = k_step / k_step_split; 'empty' / 'copy' = sk_diag floors."""
    os.environ["SK_STEP_VARIANT"] = str(variant if isinstance(variant, int) else 0)
    from skillshot_learning_amd import VecSkillshotGame
    env = VecSkillshotGame(n, seed=0, tick_limit=2000)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        env.reset(random_positions=True)
        ring = max(ring, graph_len)
        acts = env.gen_random_actions(ring)
        done = torch.empty(n, dtype=torch.uint8, device="cuda")
        o = torch.empty((2, n, 12), dtype=torch.float32, device="cuda") if obs else None
        r = torch.empty((2, n), dtype=torch.float32, device="cuda") if obs else None
    st.synchronize()
    slab = 16 * n
    sp = ctypes.c_void_p(st.cuda_stream)
    a0 = acts.data_ptr()

    planes = (ctypes.c_void_p * 6)(*[getattr(env, k).data_ptr() for k in ("pos", "rot", "qpos", "qrot", "qcdage", "misc")])
    diag = {"empty": 0, "copy": 1, "copy_xcc": 2, "copy_b8": 3}.get(variant)
    if variant == "copy_full":  # the full contract's traffic, split layout, no logic
        L = env._L
        L.skdiag_launch_full.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_int64, ctypes.c_void_p]
        with torch.cuda.stream(st):
            ob = torch.empty(26 * n, dtype=torch.float32, device="cuda")
        st.synchronize()
        obs = True

        def launch(t):
            rc = L.skdiag_launch_full(planes, ctypes.c_void_p(a0 + (t % ring) * slab), ctypes.c_void_p(done.data_ptr()),
                                      ctypes.c_void_p(ob.data_ptr()), n, sp)
            assert rc == 0
    elif diag is not None:
        L = env._L
        L.skdiag_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                    ctypes.c_void_p]

        def launch(t):
            rc = L.skdiag_launch(diag, planes, ctypes.c_void_p(a0 + (t % ring) * slab), ctypes.c_void_p(done.data_ptr()),
                                 n, sp)
            assert rc == 0
    else:
      def launch(t):
        env.step_raw(ctypes.c_void_p(a0 + (t % ring) * slab), ctypes.c_void_p(done.data_ptr()),
                     obs_ptr=None if o is None else ctypes.c_void_p(o.data_ptr()),
                     reward_ptr=None if r is None else ctypes.c_void_p(r.data_ptr()), stream=sp)

    with torch.cuda.stream(st):
        for t in range(4):
            launch(t)
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        for t in range(graph_len):
            launch(t)
    reps = max(1, steps // graph_len)
    with torch.cuda.stream(st):
        g.replay()
    st.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
    st.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (reps * graph_len)
    nb = 297 if obs else 193
    res = dict(variant=variant, envs=n, obs=obs, us_per_step=us, env_steps_per_s=n / (us * 1e-6),
               gbs=nb * n / (us * 1e-6) / 1e9, frac=nb * n / (us * 1e-6) / 8e12)
    env.close()
    del g
    return res


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variants", default="0,1")
    p.add_argument("--envs", default="65536,262144,1048576")
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--graph-len", type=int, default=200)
    p.add_argument("--ring", type=int, default=300)
    p.add_argument("--obs", action="store_true")
    a = p.parse_args()
    for v in [int(x) if x.isdigit() else x for x in a.variants.split(",")]:
        for n in [int(x) for x in a.envs.split(",")]:
            ring = a.ring if n <= 262144 else max(a.graph_len, 64)
            print(json.dumps(run(v, n, a.steps, a.graph_len, ring, obs=a.obs)), flush=True)


if __name__ == "__main__" and not os.environ.get("SWEEP_SHARDS"):
    main()


def run_sharded(n_total, shards, steps, graph_len, ring, variant=0):
    """n_total games as `shards` independent env shards on separate streams,
    each replaying its own captured chain; time for every shard to advance
    `steps` ticks."""
    os.environ["SK_STEP_VARIANT"] = str(variant)
    from skillshot_learning_amd import VecSkillshotGame
    n = n_total // shards
    envs, streams, graphs, keep = [], [], [], []
    for s in range(shards):
        env = VecSkillshotGame(n, seed=0, env_offset=s * n, tick_limit=2000)
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            env.reset(random_positions=True)
            acts = env.gen_random_actions(ring)
            done = torch.empty(n, dtype=torch.uint8, device="cuda")
        st.synchronize()
        sp = ctypes.c_void_p(st.cuda_stream)

        def launch(t, env=env, acts=acts, done=done, sp=sp):
            env.step_raw(ctypes.c_void_p(acts.data_ptr() + (t % ring) * 16 * n), ctypes.c_void_p(done.data_ptr()),
                         stream=sp)

        with torch.cuda.stream(st):
            for t in range(4):
                launch(t)
        st.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for t in range(graph_len):
                launch(t)
        envs.append(env); streams.append(st); graphs.append(g); keep.append((acts, done))
    torch.cuda.synchronize()
    reps = max(1, steps // graph_len)
    main = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(2):  # second pass is the timed one
        e0.record(main)
        for st, g in zip(streams, graphs):
            st.wait_event(e0)
            with torch.cuda.stream(st):
                for _ in range(reps):
                    g.replay()
        ends = []
        for st in streams:
            ev = torch.cuda.Event()
            ev.record(st)
            main.wait_event(ev)
        e1.record(main)
        torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (reps * graph_len)
    res = dict(variant=variant, envs=n_total, shards=shards, us_per_step=us, env_steps_per_s=n_total / (us * 1e-6),
               frac=193 * n_total / (us * 1e-6) / 8e12)
    for e in envs:
        e.close()
    return res


if __name__ == "__main__" and os.environ.get("SWEEP_SHARDS"):
    for S in [int(x) for x in os.environ["SWEEP_SHARDS"].split(",")]:
        for v in (0, 1):
            print(json.dumps(run_sharded(65536, S, 2000, 200, 300, variant=v)), flush=True)
