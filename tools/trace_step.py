"""Per-wave timeline of k_step from the -DSK_TRACE_STEP build (ab/trace.so).

    SK_LIB_PATH=ab/trace.so python tools/trace_step.py [--envs 65536] [--obs]

Graph-replays the fused step like bench.py, then reads the last 16 launches'
per-wave s_memrealtime stamps (10 ns ticks): entry, loads landed, tick done,
stores complete.  Prints one JSON line per N: dispatch ramp (spread of wave
entry), per-wave phase medians, the span from first entry to last store
completion, and the gap between one launch's last wave and the next's first.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(n, obs, G=400, ring=400):
    from skillshot_learning_amd import VecSkillshotGame
    env = VecSkillshotGame(n, seed=0, tick_limit=2000)
    L = env._L
    waves = (n + 63) // 64
    buf = torch.zeros(16 * waves * 8, dtype=torch.int64, device="cuda")
    L.skdiag_set_step_trace.argtypes = [ctypes.c_void_p]
    assert L.skdiag_set_step_trace(ctypes.c_void_p(buf.data_ptr())) == 0
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        env.reset(random_positions=True)
        acts = env.gen_random_actions(ring)
        done = torch.empty(n, dtype=torch.uint8, device="cuda")
        o = torch.empty((2, n, 12), dtype=torch.float32, device="cuda") if obs else None
    st.synchronize()
    sp = ctypes.c_void_p(st.cuda_stream)

    def launch(t):
        env.step_raw(ctypes.c_void_p(acts.data_ptr() + (t % ring) * 16 * n), ctypes.c_void_p(done.data_ptr()),
                     obs_ptr=None if o is None else ctypes.c_void_p(o.data_ptr()), stream=sp)

    with torch.cuda.stream(st):
        for t in range(4):
            launch(t)
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        for t in range(G):
            launch(t)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        g.replay()
        e0.record()
        g.replay()
        e1.record()
    st.synchronize()
    us_launch = e0.elapsed_time(e1) * 1e3 / G
    T = buf.view(16, waves, 8).cpu().numpy().astype(np.int64)
    env.close()
    order = np.argsort(T[:, :, 0].min(axis=1))
    T = T[order]
    t0, t1, t2, t3 = (T[:, :, k] * 10 for k in range(4))  # ns
    ns = lambda x: float(np.median(x))
    hw = T[0, :, 4]
    xcc = T[0, :, 5] & 0xF
    res = dict(envs=n, obs=obs, us_per_launch_event=us_launch,
               ramp_ns=ns(t0.max(1) - t0.min(1)),
               load_ns_med=ns(t1 - t0), load_ns_p90=float(np.percentile(t1 - t0, 90)),
               tick_ns_med=ns(t2 - t1), tick_ns_p90=float(np.percentile(t2 - t1, 90)),
               store_ns_med=ns(t3 - t2), store_ns_p90=float(np.percentile(t3 - t2, 90)),
               wave_ns_med=ns(t3 - t0),
               span_ns=ns(t3.max(1) - t0.min(1)),
               last_entry_to_last_done_ns=ns(t3.max(1) - t0.max(1)),
               gap_ns=ns(t0.min(1)[1:] - t3.max(1)[:-1]),
               launch_period_ns=ns(np.diff(t0.min(1))),
               # the tail: how much later than the median wave the last one finishes, and why
               end_rel_med_ns=ns(np.median(t3 - t0.min(1)[:, None], axis=1)),
               end_rel_max_ns=ns((t3 - t0.min(1)[:, None]).max(1)),
               entry_of_last_done_ns=ns((t0 - t0.min(1)[:, None])[np.arange(16), (t3).argmax(1)]),
               load_ns_max=ns((t1 - t0).max(1)), tick_ns_max=ns((t2 - t1).max(1)),
               store_ns_max=ns((t3 - t2).max(1)),
               xcc_of_wave_0_15=[int(x) for x in xcc[:16]],
               cu_ids_distinct=int(len(np.unique(hw & ~np.int64(0xF)))))
    return res


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", default="65536,262144")
    p.add_argument("--obs", action="store_true")
    a = p.parse_args()
    for n in [int(x) for x in a.envs.split(",")]:
        print(json.dumps(run(n, a.obs)), flush=True)


if __name__ == "__main__":
    main()
