"""Phase timeline of the sliced fp32 critic backward (k_grad_slice_bwd<1>:
the bootstrap critic step of configs 3-5) from a -DSK_TRACE32 build:

    tools/build_variant.sh ab_run/trace32.so -DSK_TRACE32
    SK_LIB_PATH=$PWD/ab_run/trace32.so python tools/trace_slice_bwd.py [--rows 256]

Microseconds from the first workgroup's first stamp to each phase boundary
(phase 0 = every global load, 1 = layer 1 + per-row reductions incl. the
bootstrap target, 2 = the slice's dz2, 3 = dW2 rows / dz1 share / partial
stores), first and last workgroup (s_memrealtime, 100 MHz)."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

POINTS = {20: "start", 21: "loads_staged", 22: "phase1", 23: "phase2", 24: "end"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", default="256")
    a = p.parse_args()
    from skillshot_learning_amd import learner
    d = learner.DDPG("cuda", seed=0, gamma=0.99, tau=0.005, fused_update=True, precision="fp32")
    fu = d._fused
    L = fu.L
    L.sk_debug_trace32.argtypes = [ctypes.c_void_p]
    for rows in [int(r) for r in a.rows.split(",")]:
        s = torch.rand(rows, 12, device="cuda")
        act = torch.rand(rows, 2, device="cuda") * 2 - 1
        r = torch.rand(rows, device="cuda")
        dn = torch.zeros(rows, device="cuda")
        for _ in range(6):
            fu.critic_step(s, act, s2=s, r=r, d=dn, gamma=0.99)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (2 * 32 * 2))()
        assert L.sk_debug_trace32(buf) == 0
        t = np.frombuffer(buf, dtype=np.uint64).reshape(2, 32, 2).astype(np.float64)
        t0 = min(t[0, 20, 1], t[1, 20, 1])
        out = {}
        for wg in (0, 1):
            out["first" if wg == 0 else "last"] = {n: round(float((t[wg, k, 1] - t0) / 100.0), 2)
                                                   for k, n in POINTS.items()}
        print(json.dumps({"kernel": "k_grad_slice_bwd<1>", "rows": rows, **out}), flush=True)


if __name__ == "__main__":
    main()
