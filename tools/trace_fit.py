"""Phase timeline of the resident models_fit kernels from the -DSK_TRACE_FIT
build (tools/build_variant.sh ab_run/trace_fit.so -DSK_TRACE_FIT): lane 0 of
wave 0 of every workgroup stamps 11 points of steps 64..95; prints, per
kernel, the median duration of each phase over steps and workgroups, the
median step and the spread of the step boundaries across workgroups.

    SK_LIB_PATH=$PWD/ab_run/trace_fit.so python tools/trace_fit.py

With a -DSK_TRACE_FIT -DSK_TRACE_FIT_P5 build and --p5, stamps 7 .. 9 sit
inside phase 5 (after the first products, after the first row sums / the
output, after the dz2 stores; the barrier after)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = {"critic": ["L1 + Dropout", "P1 publish", "R sum + H publish", "H gather", "q + dz2", "dh1 GEMM",
                    "dW1 + Adam (waves 2/3: unit Adam)", "-", "dW2 GEMM + Adam", "-", "to the next step"],
         "actor": ["L1 x2", "P1 publish x2", "R sums + H publish", "H gather", "a, dQ/da, dz2", "dh1 GEMM",
                   "dW1 + Adam (waves 2/3: unit Adam)", "-", "dW2 GEMM + Adam", "-", "to the next step"]}


P5_NAMES = {"critic": ["L1 + Dropout", "P1 publish", "R sum + H publish", "H gather", "5a: W3 h2 products",
                       "5b: q row sum, dq", "5c: dz2 stores", "5d: barrier", "dh1 GEMM", "dW1 + dW2 + Adam",
                       "to the next step"],
            "actor": ["L1", "P1 publish", "R sums + H publish", "H gather", "5a: W3 h2 products",
                      "5b: row sums, tanh, critic dQ/da products", "5c: row sums, dz2 stores", "5d: barrier",
                      "dh1 GEMM", "dW1 + dW2 + Adam", "to the next step"]}
P5_ORDER = [0, 1, 2, 3, 4, 7, 8, 9, 5, 6, 10]


def main():
    p5 = "--p5" in sys.argv
    from skillshot_learning_amd import learner
    dev = torch.device("cuda", 0)
    d = learner.DDPG("cuda", seed=0, fused_update=True, precision="fp32")
    fu = d._fused
    fu.soft_update_in_adam = False
    L = fu.L
    L.skdiag_set_fit_trace.argtypes = [ctypes.c_void_p]
    P = int(os.environ.get("SK_FIT_P", "16"))
    buf = torch.zeros(P * 32 * 12, dtype=torch.int64, device=dev)
    assert L.skdiag_set_fit_trace(ctypes.c_void_p(buf.data_ptr())) == 0
    n = 256
    g = torch.Generator(device=dev).manual_seed(1)
    S = torch.rand(16 * n, 12, device=dev, generator=g)
    A = torch.rand(16 * n, 2, device=dev, generator=g) * 2 - 1
    R = torch.randn(16 * n, device=dev, generator=g)
    fu.FIT_STEPS_PER_LAUNCH = n
    out = {}
    for kind, fn in (("critic", lambda: fu.fit_critic(S, A, R)), ("actor", lambda: fu.fit_actor(S))):
        fn()
        buf.zero_()
        fn()
        torch.cuda.synchronize()
        fu.fit_check()
        ts = buf.view(P, 32, 12).cpu().numpy().astype(np.int64)
        if p5:
            ts = ts[:, :, P5_ORDER + [11]]
        ph = np.diff(ts[:, :, :11], axis=2) * 0.01  # us: phases 0..9
        tail = np.zeros_like(ph[:, :, :1])
        tail[:, :-1, 0] = (ts[:, 1:, 0] - ts[:, :-1, 10]) * 0.01  # stamp 10 to the next step's 0
        tail[:, -1, 0] = tail[:, -2, 0]
        ph = np.concatenate([ph, tail], axis=2)
        step = (ts[:, 1:, 0] - ts[:, :-1, 0]) * 0.01
        out[kind] = dict(step_us_p50=round(float(np.median(step)), 3),
                         phases_us_p50={nm: round(float(np.median(ph[:, :, i])), 3) for i, nm in enumerate((P5_NAMES if p5 else NAMES)[kind])},
                         phases_us_max={nm: round(float(np.max(np.median(ph[:, :, i], axis=1))), 3)
                                        for i, nm in enumerate((P5_NAMES if p5 else NAMES)[kind])},
                         step_start_spread_us_p50=round(float(np.median(ts[:, :, 0].max(0) - ts[:, :, 0].min(0))) * 0.01, 3))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
