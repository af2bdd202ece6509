"""Phase timeline of the fused update kernels (k_critic_grad with the
in-kernel bootstrap target, k_actor_grad) from a -DSK_TRACE build:

    hipcc ... -DSK_TRACE -o ab/trace.so <sources>   (see tools/README.md)
    SK_LIB_PATH=$PWD/ab/trace.so python tools/trace_update.py [--rows 256,4096]

Prints, per kernel and batch, the microseconds from the kernel's first
timestamp to each trace point for the first and the last workgroup
(s_memtime deltas scaled by the wall-clock rate measured between the
first and last points).
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CRITIC = ["start", "init", "staged", "layer1x3", "layer2x2", "q_mu_targetQ", "y_dz2", "backward", "store_partials",
          "end"]
ACTOR = ["start", "init", "staged", "layer1x2", "layer2x2", "mu_critic_dq", "dz3_dz2", "backward", "store_partials",
         "end"]


def read(L):
    buf = (ctypes.c_ulonglong * (2 * 32 * 2))()
    assert L.sk_debug_update_trace(buf) == 0
    return np.frombuffer(buf, dtype=np.uint64).reshape(2, 32, 2).astype(np.float64)


def timeline(t, names):
    out = {}
    for wg in (0, 1):
        mt, rt = t[wg, :len(names), 0], t[wg, :len(names), 1]
        rate = (mt[-1] - mt[0]) / max(rt[-1] - rt[0], 1)  # memtime ticks per 10 ns
        us = (mt - mt[0]) / rate / 100.0 if rate > 0 else (rt - rt[0]) / 100.0
        d = {n: round(float(u), 2) for n, u in zip(names, us)}
        # optional sub-phase points 12..15 (diagnostic builds that set them)
        extra = t[wg, 12:16, 0]
        if rate > 0 and (extra > 0).all():
            d.update({f"tp{12 + k}": round(float((x - mt[0]) / rate / 100.0), 2) for k, x in enumerate(extra)})
        out["first" if wg == 0 else "last"] = d
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", default="256,4096")
    a = p.parse_args()
    from skillshot_learning_amd import learner, _capi
    ddpg = learner.DDPG("cuda", seed=0, fused_update=True, precision="bf16")
    fu = ddpg._fused
    L = fu.L
    L.sk_debug_update_trace.argtypes = [ctypes.c_void_p]
    for rows in [int(r) for r in a.rows.split(",")]:
        s = torch.rand(rows, 12, device="cuda")
        act = torch.rand(rows, 2, device="cuda") * 2 - 1
        r = torch.rand(rows, device="cuda")
        d = torch.zeros(rows, device="cuda")
        for name, fn, names in (
                ("critic_grad_bootstrap", lambda: fu.grads("critic", s, act, None, None, s, r, d, 0.99), CRITIC),
                ("actor_grad", lambda: fu.grads("actor", s), ACTOR)):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            fn()
            torch.cuda.synchronize()
            print(json.dumps({"kernel": name, "rows": rows, **timeline(read(L), names)}), flush=True)


if __name__ == "__main__":
    main()
