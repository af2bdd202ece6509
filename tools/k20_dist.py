"""Distribution of the driver's K = 20 headline region (bench.timed_multi at
--steps 20 --warmup 5) over many repetitions in one process: per rep the
400-slab action ring is generated afresh (so the cache holds what it holds
after bench's own generation), 1 + 5 warm-up ticks run, then ONE 20-tick
k_step_multi launch is timed with HIP events on its stream.  The driver runs
this region once per bench; its event time varies by a few percent from run
to run, so library A/Bs of the headline compare medians over reps here.

    SK_LIB_PATH=... python tools/k20_dist.py [--reps 40] [--k 20] [--warmup 5]
prints one JSON line: median / mean / p10 / p90 event us per tick and frac.
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
    p.add_argument("--reps", type=int, default=40)
    p.add_argument("--k", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--envs", type=int, default=65536)
    p.add_argument("--tag", default=os.path.basename(os.environ.get("SK_LIB_PATH", "lib")))
    p.add_argument("--settle", choices=["none", "sweep", "long", "heat", "long_reset"], default="none",
                   help="between the ring's generation and the warm-up: nothing (bench), a 512 MiB read "
                        "sweep of another buffer (evicts the generation's dirty lines from the Infinity "
                        "Cache), 400 more warm-up ticks (a long run's cache state), a ~3 ms matmul before the ring's "
                        "generation (clocks), or 400 ticks then the env reset and the ring regenerated")
    p.add_argument("--stream", choices=["side", "default"], default="side",
                   help="launch on bench's side stream or on the default (null) stream")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    n, ring = a.envs, 400
    env, st, acts = bench._env_and_actions(dev, n, 0, 0, 2000, ring)
    if a.stream == "default":
        st = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    done = torch.empty(n, dtype=torch.uint8, device=dev)
    ap, dp = ctypes.c_void_p(acts.data_ptr()), ctypes.c_void_p(done.data_ptr())
    fn, h, lim, rp = env._L.sk_env_step_multi, env._h, env.tick_limit, int(env.random_positions)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    e1.record(st)
    us, wall = [], []
    big = torch.ones(128 << 20, dtype=torch.float32, device=dev) if a.settle == "sweep" else None
    sink = torch.zeros((), dtype=torch.float32, device=dev)
    mm = torch.randn(4096, 4096, device=dev) if a.settle == "heat" else None
    for rep in range(a.reps + 1):
        with torch.cuda.stream(st):
            if a.settle == "heat":
                sink.add_((mm @ mm).sum() + (mm @ mm).sum())
            if a.settle == "long_reset":
                fn(h, ap, ring, 0, 400, dp, None, 0, lim, 1, rp, sp)
            env.reset(random_positions=True)
            acts.copy_(env.gen_random_actions(ring))  # the ring rewritten: bench's cache state
        slab = 0
        if a.settle == "sweep":
            with torch.cuda.stream(st):
                sink.add_(big.sum())
        elif a.settle == "long":
            fn(h, ap, ring, 0, 400, dp, None, 0, lim, 1, rp, sp)
            slab = 400 % ring
        for t in (1, a.warmup):
            fn(h, ap, ring, slab, t, dp, None, 0, lim, 1, rp, sp)
            slab += t
        st.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(st)
        fn(h, ap, ring, slab, a.k, dp, None, 0, lim, 1, rp, sp)
        e1.record(st)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if rep:  # the first rep loads code objects
            us.append(e0.elapsed_time(e1) * 1e3 / a.k)
            wall.append(el * 1e6 / a.k)
    us.sort()
    q = lambda f: us[min(len(us) - 1, int(f * len(us)))]  # noqa: E731
    med = statistics.median(us)
    print(json.dumps(dict(tag=a.tag, settle=a.settle, stream=a.stream, wall_us_median=round(statistics.median(wall), 4), k=a.k, reps=a.reps, event_us_median=round(med, 4),
                          event_us_mean=round(statistics.fmean(us), 4), p10=round(q(0.1), 4), p90=round(q(0.9), 4),
                          frac_median=round(193 * n / (med * 1e-6) / 8e12, 4))), flush=True)
    env.close()


if __name__ == "__main__":
    main()
