"""Per-wave timeline of k_step_multi from the -DSK_TRACE_MULTI build
(ab/trace_multi.so): where a short launch's fixed cost goes.

    SK_LIB_PATH=ab/trace_multi.so python tools/trace_multi.py [--envs 65536] [--ticks 20]

Runs the bench's launch pattern (one warm-up launch, then timed launches of
--ticks ticks on a 400-slab action ring) and reads the last launch's stamps
(10 ns): per wave entry, end of ticks 0..29, exit.  Prints one JSON line:
entry spread, per-tick medians and maxima over waves (tick 0 holds the cold
start), the exit spread and the span first entry -> last exit."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=65536)
    p.add_argument("--ticks", type=int, default=20)
    p.add_argument("--launches", type=int, default=5)
    a = p.parse_args()
    from skillshot_learning_amd import VecSkillshotGame
    n, T = a.envs, a.ticks
    env = VecSkillshotGame(n, seed=0, tick_limit=2000)
    L = env._L
    waves = (n + 63) // 64
    buf = torch.zeros(waves * 32, dtype=torch.int64, device="cuda")
    L.skdiag_set_multi_trace.argtypes = [ctypes.c_void_p]
    assert L.skdiag_set_multi_trace(ctypes.c_void_p(buf.data_ptr())) == 0
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        env.reset(random_positions=True)
        acts = env.gen_random_actions(400)
        done = torch.empty(n, dtype=torch.uint8, device="cuda")
        win = torch.empty(n, dtype=torch.uint8, device="cuda")
    st.synchronize()
    sp = ctypes.c_void_p(st.cuda_stream)
    slab = 0
    out = []
    for k in range(a.launches):
        env.step_multi_raw(ctypes.c_void_p(acts.data_ptr()), 400, slab, T if k else 5,
                           ctypes.c_void_p(done.data_ptr()), ctypes.c_void_p(win.data_ptr()), stream=sp)
        slab = (slab + (T if k else 5)) % 400
        st.synchronize()
        if k == 0:
            continue
        ts = buf.view(waves, 32).cpu().numpy().astype(np.int64)
        t0 = ts[:, 0].min()
        e = ts[:, 0] - t0
        nt = min(T, 30)
        ends = ts[:, 1:1 + nt] - t0
        per = np.diff(np.concatenate([ts[:, :1] - t0, ends], axis=1), axis=1) * 10 / 1e3  # us
        x = ts[:, 31] - t0
        out.append(dict(entry_spread_us=float(e.max() - e.min()) * 0.01, entry_p50_us=float(np.median(e)) * 0.01,
                        tick_p50_us=[round(float(v), 3) for v in np.median(per, axis=0)],
                        tick_max_us=[round(float(v), 3) for v in per.max(axis=0)],
                        last_tick_to_exit_p50_us=float(np.median(x - ends[:, -1])) * 0.01,
                        exit_min_us=float(x.min()) * 0.01, exit_p50_us=float(np.median(x)) * 0.01,
                        span_us=float(x.max()) * 0.01))
    print(json.dumps(dict(envs=n, ticks=T, launches=out[-2:])))


if __name__ == "__main__":
    main()
