"""The driver's short timed region (bench.timed_multi: two events around one
k_step_multi launch of K ticks, then torch.cuda.synchronize) on a side
stream (bench.py's) against the same region on the default stream, and the
cost of the synchronize calls themselves on an idle GPU.  Medians over reps.

    python tools/short_run_streams.py [--k 20] [--reps 40]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--k", type=int, default=20)
    p.add_argument("--reps", type=int, default=40)
    p.add_argument("--envs", type=int, default=65536)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    ring = 400
    env, side, acts = bench._env_and_actions(dev, a.envs, 0, 0, 2000, ring)
    done = torch.empty(a.envs, dtype=torch.uint8, device=dev)
    ap, dp = ctypes.c_void_p(acts.data_ptr()), ctypes.c_void_p(done.data_ptr())
    fn, h, lim, rp = env._L.sk_env_step_multi, env._h, env.tick_limit, int(env.random_positions)
    default = torch.cuda.default_stream(dev)
    rows = {}
    slab = 0

    def add(k, v):
        rows.setdefault(k, []).append(v)

    for st, name in ((side, "side"), (default, "default")):
        sp = ctypes.c_void_p(st.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        e1.record(st)
        for _ in range(5):
            assert fn(h, ap, ring, slab, a.k, dp, None, 0, lim, 1, rp, sp) == 0
        torch.cuda.synchronize()
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(st)
            assert fn(h, ap, ring, slab, a.k, dp, None, 0, lim, 1, rp, sp) == 0
            e1.record(st)
            torch.cuda.synchronize()
            add(f"wall_{name}", (time.perf_counter() - t0) * 1e6)
            add(f"event_{name}", e0.elapsed_time(e1) * 1e3)
            slab = (slab + a.k) % ring
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            torch.cuda.synchronize()
            add("idle_device_sync", (time.perf_counter() - t0) * 1e6)
            t0 = time.perf_counter()
            st.synchronize()
            add(f"idle_stream_sync_{name}", (time.perf_counter() - t0) * 1e6)
            t0 = time.perf_counter()
            e1.record(st)
            e1.synchronize()
            add(f"idle_event_roundtrip_{name}", (time.perf_counter() - t0) * 1e6)
    out = {k: round(statistics.median(v), 2) for k, v in rows.items()}
    out.update(k=a.k, envs=a.envs, unit="us (median over reps)")
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
