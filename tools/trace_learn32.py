"""Phase timeline of k_critic_grad32 (fp32 critic step with the in-launch
bootstrap target) from a -DSK_TRACE32 build of libskillshot:

    tools/build_variant.sh ab/trace32.so -DSK_TRACE32
    SK_LIB_PATH=$PWD/ab/trace32.so python tools/trace_learn32.py [--rows 256,4096]

Microseconds from the kernel's first timestamp to each trace point, first and
last workgroup."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CRITIC = ["start", "staged", "layer1x3", "layer2x2", "targetQ", "y_dz2", "dW2_dz1", "dW1", "store_partials",
          "end"]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", default="256,4096")
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
            fu.grads("critic", s, act, s2=s, r=r, d=dn, gamma=0.99)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (2 * 32 * 2))()
        assert L.sk_debug_trace32(buf) == 0
        t = np.frombuffer(buf, dtype=np.uint64).reshape(2, 32, 2).astype(np.float64)
        out = {}
        for wg in (0, 1):
            rt = t[wg, :len(CRITIC), 1]
            out["first" if wg == 0 else "last"] = {n: round(float((x - rt[0]) / 100.0), 2) for n, x in zip(CRITIC, rt)}
        print(json.dumps({"kernel": "k_critic_grad32", "rows": rows, **out}), flush=True)


if __name__ == "__main__":
    main()
