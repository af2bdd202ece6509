"""Diagnose future-collision (A11) mismatches between the HIP features kernel
and the reference probes (tests/golden/probes.npz): per mismatch, the device
and libm gradients (ulp distance) and the boundary compare with and without a
fused multiply-add."""
import math
import os
import sys
from fractions import Fraction

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import golden_replay as gr  # noqa: E402
import skillshot_learning_amd as ssa  # noqa: E402

d = gr.load("probes")
n = d["pos"].shape[0]
g = ssa.VecSkillshotGame(n)
g.load_state_dict(gr.probe_state(d))
f = g.features().cpu().numpy()
bad = np.argwhere(f[..., 17].astype(np.uint8) != d["future"])
gd_all = f[..., 8]
gc_all = np.array([[math.tan(-d["qrot"][i, p] + math.pi / 2) for p in (0, 1)] for i in range(n)])
ulp = np.abs(gd_all.view(np.int64) - gc_all.view(np.int64))
print(f"mismatches {len(bad)} / {2 * n}; gradient ulp hist: "
      f"0:{int((ulp == 0).sum())} 1:{int((ulp == 1).sum())} >1:{int((ulp > 1).sum())}")
for i, p in bad[:40]:
    qx, qy = (int(v) for v in d["qpos"][i, p])
    ox, oy = (int(v) for v in d["pos"][i, 1 - p])
    gd, gc = float(gd_all[i, p]), float(gc_all[i, p])
    yi = float(qy) - gc * float(qx)
    yi_f = float(Fraction(qy) - Fraction(gc) * qx)
    res = []
    for X in (ox, ox + 5):
        v = gc * float(X) + yi
        vf = float(Fraction(gc) * X + Fraction(yi_f))
        vfd = float(Fraction(gd) * X + Fraction(float(Fraction(qy) - Fraction(gd) * qx)))
        res.append((v, vf, vfd))
    print(i, p, "rot", repr(d["qrot"][i, p]), "ulp", int(ulp[i, p]), "want", d["future"][i, p],
          "got", f[i, p, 17], "oy", oy, [(repr(a), repr(b), repr(c)) for a, b, c in res])
