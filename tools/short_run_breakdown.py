"""Where the ~30 us of fixed wall time in a 20-step timed region goes:
host time of the graph launch call, time until the last event is seen
complete by a busy poll, and the synchronize after it, against the HIP-event
span of the same region (bench.py's TickGraphs, 65,536 games).

    python tools/short_run_breakdown.py [--k 20] [--reps 30]
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
    p.add_argument("--reps", type=int, default=30)
    p.add_argument("--envs", type=int, default=65536)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    n = a.envs
    env, st, acts = bench._env_and_actions(dev, n, 0, 0, 2000, 400)
    slab, sp = 16 * n, ctypes.c_void_p(st.cuda_stream)
    done = torch.empty(n, dtype=torch.uint8, device=dev)
    a0, dp = acts.data_ptr(), ctypes.c_void_p(done.data_ptr())

    def launch(t):
        env.step_raw(ctypes.c_void_p(a0 + (t % 400) * slab), dp, stream=sp)

    with torch.cuda.stream(st):
        for t in range(4):
            launch(t)
    st.synchronize()
    tg = bench.TickGraphs(env, st, launch, 400)
    tg.prepare(a.k)
    rows = {k: [] for k in ("launch_call", "poll_done", "sync_after_poll", "wall", "event", "wall_plain")}
    for rep in range(a.reps):
        tg.sync()
        st.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(st):
            e0.record()
        tg.replay(a.k)
        t1 = time.perf_counter()
        with torch.cuda.stream(st):
            e1.record()
        while not e1.query():
            pass
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        rows["launch_call"].append((t1 - t0) * 1e6)
        rows["poll_done"].append((t2 - t0) * 1e6)
        rows["sync_after_poll"].append((t3 - t2) * 1e6)
        rows["wall"].append((t3 - t0) * 1e6)
        rows["event"].append(e0.elapsed_time(e1) * 1e3)
        # the same region exactly as bench.py times it (events, blocking synchronize)
        tg.sync()
        st.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(st):
            e0.record()
        tg.replay(a.k)
        with torch.cuda.stream(st):
            e1.record()
        torch.cuda.synchronize()
        rows["wall_plain"].append((time.perf_counter() - t0) * 1e6)
    out = {k: round(statistics.median(v), 2) for k, v in rows.items()}
    out.update(k=a.k, envs=n, unit="us (median over reps)")
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
