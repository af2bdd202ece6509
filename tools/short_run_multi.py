"""Where the fixed wall time of a short timed region goes with the multi-tick
headline (bench.timed_multi: K ticks in one k_step_multi launch): host time
of each call in the region, the time until a busy poll sees the last event
complete, and the synchronize after it, against the HIP-event span.  Also
the same region with the launch made straight through the pre-bound ctypes
function (no Python wrapper) and with a stream instead of a device
synchronize.

    python tools/short_run_multi.py [--k 20] [--reps 30]
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
    n, ring = a.envs, 400
    env, st, acts = bench._env_and_actions(dev, n, 0, 0, 2000, ring)
    sp = ctypes.c_void_p(st.cuda_stream)
    done = torch.empty(n, dtype=torch.uint8, device=dev)
    ap, dp = ctypes.c_void_p(acts.data_ptr()), ctypes.c_void_p(done.data_ptr())
    fn = env._L.sk_env_step_multi
    h = env._h

    def launch_py():
        env.step_multi_raw(ap, ring, 0, a.k, dp, None, 0, stream=sp)

    def launch_direct():
        fn(h, ap, ring, 0, a.k, dp, None, 0, 2000, 1, 1, sp)

    launch_py()
    st.synchronize()
    rows = {}

    def add(k, v):
        rows.setdefault(k, []).append(v)

    for rep in range(a.reps):
        # 1) bench's region, instrumented
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(st):
            e0.record()
        t1 = time.perf_counter()
        launch_py()
        t2 = time.perf_counter()
        with torch.cuda.stream(st):
            e1.record()
        t3 = time.perf_counter()
        while not e1.query():
            pass
        t4 = time.perf_counter()
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        add("rec0_call", (t1 - t0) * 1e6)
        add("launch_call_py", (t2 - t1) * 1e6)
        add("rec1_call", (t3 - t2) * 1e6)
        add("poll_done", (t4 - t0) * 1e6)
        add("sync_after_poll", (t5 - t4) * 1e6)
        add("event", e0.elapsed_time(e1) * 1e3)
        # 2) bench's region as is
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(st):
            e0.record()
        launch_py()
        with torch.cuda.stream(st):
            e1.record()
        torch.cuda.synchronize()
        add("wall_bench", (time.perf_counter() - t0) * 1e6)
        add("event_bench", e0.elapsed_time(e1) * 1e3)
        # 3) direct ctypes launch, events, device sync
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(st)
        launch_direct()
        e1.record(st)
        torch.cuda.synchronize()
        add("wall_direct", (time.perf_counter() - t0) * 1e6)
        add("event_direct", e0.elapsed_time(e1) * 1e3)
        # 4) direct launch, no events, stream sync
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        launch_direct()
        st.synchronize()
        add("wall_direct_noevents_streamsync", (time.perf_counter() - t0) * 1e6)
        # 5) an empty region (sync only)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(st)
        e1.record(st)
        torch.cuda.synchronize()
        add("wall_events_only", (time.perf_counter() - t0) * 1e6)
    out = {k: round(statistics.median(v), 2) for k, v in rows.items()}
    out.update(k=a.k, envs=n, unit="us (median over reps)")
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
