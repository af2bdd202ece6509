"""Where the fixed cost of a SHORT timed region goes (the driver runs bench.py
with --steps 20): K graph-replayed k_step launches at 65,536 games, timed as
bench.py times them (barrier-free N=1: synchronize, perf_counter, replay,
synchronize), per launch method:

  torch     torch.cuda.CUDAGraph.replay() of a K-node graph (bench.py today)
  direct    hipGraphLaunch of the same executable graph through ctypes
  eager     K ctypes launches, no graph
and, with --idle-us, a busy pre-kernel before the timed region (is the first
launch after an idle GPU slow?).  One JSON line per method with wall and
HIP-event microseconds per step (median of --reps).  Run under different
environments (e.g. DEBUG_CLR_GRAPH_PACKET_CAPTURE) in separate processes.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from skillshot_learning_amd import VecSkillshotGame  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--k", type=int, default=20)
    p.add_argument("--reps", type=int, default=15)
    p.add_argument("--envs", type=int, default=65536)
    p.add_argument("--spin", action="store_true", help="hipSetDeviceFlags(hipDeviceScheduleSpin) before the device is used")
    a = p.parse_args()
    if a.spin:
        hp = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
        rc = ctypes.CDLL(hp).hipSetDeviceFlags(ctypes.c_uint(1))
        print(json.dumps(dict(spin_rc=rc)), flush=True)
    n, K = a.envs, a.k
    g = VecSkillshotGame(n, device="cuda:0", seed=0, random_positions=True)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        g.reset(random_positions=True)
        acts = g.gen_random_actions(K)
        done = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    st.synchronize()
    sp = ctypes.c_void_p(st.cuda_stream)

    def launch(t):
        g.step_raw(ctypes.c_void_p(acts.data_ptr() + (t % K) * 16 * n), ctypes.c_void_p(done.data_ptr()), stream=sp)

    with torch.cuda.stream(st):
        for t in range(4):
            launch(t)
    g.sync_step_counter(sp)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=st):
        for t in range(K):
            launch(t)
    st.synchronize()
    path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
    hip = ctypes.CDLL(path)
    hip.hipGraphLaunch.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    ex = ctypes.c_void_p(gr.raw_cuda_graph_exec())
    hip.hipGraphUpload(ex, sp)
    st.synchronize()

    cur = {}

    def run(method):
        if method == "torch":
            with torch.cuda.stream(st):
                cur["gr"].replay()
        elif method == "direct":
            hip.hipGraphLaunch(cur["ex"], sp)
        else:
            with torch.cuda.stream(st):
                for t in range(K):
                    launch(t)

    env = {k: v for k, v in os.environ.items() if k.startswith(("DEBUG_CLR", "HIP_", "GPU_", "ROC_"))}
    env["spin"] = a.spin
    for method in ("torch", "direct", "eager"):
        gr = torch.cuda.CUDAGraph()
        g.sync_step_counter(sp)
        with torch.cuda.graph(gr, stream=st):
            for t in range(K):
                launch(t)
        ex = ctypes.c_void_p(gr.raw_cuda_graph_exec())
        cur.update(gr=gr, ex=ex)
        if os.environ.get("SK_NO_UPLOAD") != "1":
            hip.hipGraphUpload(ex, sp)
        st.synchronize()
        walls, evs = [], []
        for r in range(a.reps):
            g.sync_step_counter(sp)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with torch.cuda.stream(st):
                e0.record()
            run(method)
            with torch.cuda.stream(st):
                e1.record()
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e6 / K)
            evs.append(e0.elapsed_time(e1) * 1e3 / K)
        first_wall, first_ev = walls[0], evs[0]
        walls, evs = walls[1:], evs[1:]
        walls.sort()
        evs.sort()
        print(json.dumps(dict(method=method, k=K, envs=n, first_wall_us=first_wall, first_event_us=first_ev,
                              wall_us_per_step=walls[len(walls) // 2],
                              event_us_per_step=evs[len(evs) // 2], wall_min=walls[0], env=env)), flush=True)


if __name__ == "__main__":
    main()
