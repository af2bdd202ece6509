"""Per-wave timeline of k_step_multi from the -DSK_TRACE_MULTI build
(ab/trace_multi.so): where a short launch's fixed cost goes.

    SK_LIB_PATH=ab/trace_multi.so python tools/trace_multi.py [--envs 65536] [--ticks 20]

Runs the bench's launch pattern (one warm-up launch, then timed launches of
--ticks ticks on a 400-slab action ring) and reads the last launch's stamps
(10 ns): per wave entry, end of ticks 0..28, exit, and its hardware slot (XCC,
SE, CU, SIMD: waves sharing a SIMD, their spans and exits).  Prints one JSON line:
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
    p.add_argument("--dump", default="", help="save the last launch's raw stamps [waves][32] (.npy)")
    p.add_argument("--wait", action="store_true",
                   help="the -DSK_TRACE_MULTI_WAIT build: per tick 0..4 five stamps -> issue (+ carry) / load wait / "
                        "tick_env / done + reset / state store medians")
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
        if a.dump and k == a.launches - 1:
            np.save(a.dump, ts)
        t0 = ts[:, 0].min()
        e = ts[:, 0] - t0
        if a.wait:
            nt = min(T, 5)
            st5 = (ts[:, 1:1 + 5 * nt].reshape(-1, nt, 5) - t0) * 0.01  # us
            prev = np.concatenate([e[:, None] * 0.01, st5[:, :-1, 4]], axis=1)
            parts = dict(issue=st5[:, :, 0] - prev, wait=st5[:, :, 1] - st5[:, :, 0],
                         tick=st5[:, :, 2] - st5[:, :, 1], done_reset=st5[:, :, 3] - st5[:, :, 2],
                         store=st5[:, :, 4] - st5[:, :, 3])
            out.append({k + "_p50_us": [round(float(v), 3) for v in np.median(x, axis=0)] for k, x in parts.items()}
                       | {k + "_p90_us": [round(float(v), 3) for v in np.quantile(x, 0.9, axis=0)]
                          for k, x in parts.items()})
            continue
        nt = min(T, 29)
        ends = ts[:, 1:1 + nt] - t0
        per = np.diff(np.concatenate([ts[:, :1] - t0, ends], axis=1), axis=1) * 10 / 1e3  # us
        x = ts[:, 31] - t0
        hw = ts[:, 30].astype(np.uint64)
        hwid, xcc = hw & np.uint64(0xffffffff), hw >> np.uint64(32)
        simd = (hwid >> np.uint64(4)) & np.uint64(3)
        cu = (hwid >> np.uint64(8)) & np.uint64(15)
        sh = (hwid >> np.uint64(12)) & np.uint64(1)
        se = (hwid >> np.uint64(13)) & np.uint64(7)
        slot = (((xcc * np.uint64(8) + se) * np.uint64(2) + sh) * np.uint64(16) + cu) * np.uint64(4) + simd
        _, inv, cnt = np.unique(slot, return_inverse=True, return_counts=True)
        share = cnt[inv]  # waves of this launch on the same SIMD
        cuslot = slot // np.uint64(4)
        _, cinv, ccnt = np.unique(cuslot, return_inverse=True, return_counts=True)
        span_w = (x - e) * 0.01
        out.append(dict(simds_used=int(len(cnt)), waves_per_simd_hist={int(k): int((cnt == k).sum()) for k in np.unique(cnt)},
                        cus_used=int(len(ccnt)), waves_per_cu_hist={int(k): int((ccnt == k).sum()) for k in np.unique(ccnt)},
                        xcc_hist={int(k): int((xcc == k).sum()) for k in np.unique(xcc)},
                        wave_span_us_by_share={int(k): round(float(np.median(span_w[share == k])), 3) for k in np.unique(share)},
                        exit_us_by_share={int(k): round(float(np.max(x[share == k])) * 0.01, 3) for k in np.unique(share)},
                        entry_spread_us=float(e.max() - e.min()) * 0.01, entry_p50_us=float(np.median(e)) * 0.01,
                        tick_p50_us=[round(float(v), 3) for v in np.median(per, axis=0)],
                        tick_max_us=[round(float(v), 3) for v in per.max(axis=0)],
                        last_tick_to_exit_p50_us=float(np.median(x - ends[:, -1])) * 0.01,
                        exit_min_us=float(x.min()) * 0.01, exit_p50_us=float(np.median(x)) * 0.01,
                        span_us=float(x.max()) * 0.01,
                        # is the slow-wave tail systematic? per XCD: exit p50 / max, wave span p50 / max,
                        # mean per-tick time, entry p50 (us)
                        by_xcc={int(k): dict(exit_p50=round(float(np.median(x[xcc == k])) * 0.01, 2),
                                             exit_max=round(float(np.max(x[xcc == k])) * 0.01, 2),
                                             span_p50=round(float(np.median(span_w[xcc == k])), 2),
                                             span_max=round(float(np.max(span_w[xcc == k])), 2),
                                             tick_mean=round(float(per[xcc == k].mean()), 3),
                                             entry_p50=round(float(np.median(e[xcc == k])) * 0.01, 2))
                                for k in np.unique(xcc)},
                        # the slowest 5 % of waves: their XCD and CU-slot spread
                        slow_waves_xcc_hist={int(k): int(v) for k, v in zip(*np.unique(
                            xcc[span_w >= np.quantile(span_w, 0.95)], return_counts=True))}))
    print(json.dumps(dict(envs=n, ticks=T, launches=out[-2:])))


if __name__ == "__main__":
    main()
