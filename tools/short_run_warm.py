"""Why is the first timed region of a short bench run (the driver's --steps 20
--warmup 5) slower per step than a steady one?  Repeats bench.timed_ticks'
setup (fresh env, action ring, chunk/remainder graph capture, W warmup
launches) and times the K-launch region under variants, interleaved:

  base      bench.py as it is
  idle      20 ms host sleep between the warmup and the timed region
  busy      ~3 ms of unrelated GPU work right before the warmup
  warmexec  the timed graph launched once before the warmup (exec not cold)
  smallring the action ring only K slabs (cache-resident actions)
  chunkC    graphs of C launches (C even), so the W warmup launches replay
            the chunk graph the timed region replays K/C times

One JSON line per (variant, rep): wall and HIP-event us per step.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def one(dev, variant, n, K, W, ring, chunk):
    env, st, acts = bench._env_and_actions(dev, n, 0, 0, 2000, K if variant == "smallring" else ring)
    slab, sp = 16 * n, ctypes.c_void_p(st.cuda_stream)
    done = torch.empty(n, dtype=torch.uint8, device=dev)
    a0, dp = acts.data_ptr(), ctypes.c_void_p(done.data_ptr())
    rr = K if variant == "smallring" else ring

    def launch(t):
        env.step_raw(ctypes.c_void_p(a0 + (t % rr) * slab), dp, stream=sp)

    with torch.cuda.stream(st):
        for t in range(4):
            launch(t)
    st.synchronize()
    if variant.startswith("chunk"):  # chunkC: graphs of C launches, the warmup replays the same chunk graph
        chunk = int(variant[5:])
    tg = bench.TickGraphs(env, st, launch, chunk)
    tg.prepare(W)
    tg.prepare(K)
    if variant == "warmexec":
        tg.sync()
        tg.replay(K)
        st.synchronize()
    if variant == "busy":
        x = torch.randn(4096, 4096, device=dev)
        for _ in range(20):
            x = x @ x
            x = x / x.norm()
    tg.sync()
    tg.replay(W)
    tg.sync()
    st.synchronize()
    if variant == "idle":
        time.sleep(0.02)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(st):
        e0.record()
    tg.replay(K)
    with torch.cuda.stream(st):
        e1.record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ev = e0.elapsed_time(e1)
    del tg
    env.close()
    return el * 1e6 / K, ev * 1e3 / K


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--k", type=int, default=20)
    p.add_argument("--w", type=int, default=5)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--envs", type=int, default=65536)
    p.add_argument("--variants", default="base,warmexec,chunk4,chunk2,chunk10")
    a = p.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    for r in range(a.reps):
        for v in a.variants.split(","):
            w, e = one(dev, v, a.envs, a.k, a.w, 400, 400)
            print(json.dumps(dict(variant=v, rep=r, k=a.k, w=a.w, wall_us_per_step=w, event_us_per_step=e)),
                  flush=True)


if __name__ == "__main__":
    main()
