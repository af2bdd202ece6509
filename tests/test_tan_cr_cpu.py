"""csrc/sk_tan_cr.hpp compiled for the host (same -ffp-contract=off as the
kernels; the device evaluates the same IEEE operations, fma = v_fma_f64)
against a 70-digit Decimal tan: every result correctly rounded.  The
arguments are the game's tan inputs -rot + pi/2 over the rotation ranges
play reaches, multiples of pi/4 (gradients 0, +-1, ~1.6e16) and near them."""
import math
import os
import subprocess

import numpy as np

from cr_tan import cr_tan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _args(n, seed=0):
    rng = np.random.default_rng(seed)
    rot = np.concatenate([
        rng.uniform(-math.pi, math.pi, n // 4),
        rng.uniform(-60, 60, n // 4),
        rng.uniform(-1000, 1000, n // 8),
        np.arange(-64, 65) * (math.pi / 4),
        np.arange(-64, 65) * (math.pi / 4) + rng.choice([-1e-15, 1e-15, -1e-12, 1e-9], 129),
        np.arange(-40, 41) * 0.25,  # discrete look steps (Player.py:27-31)
        rng.uniform(-1e-6, 1e-6, 64),
    ])
    return -rot + math.pi / 2


def test_tan_cr_is_correctly_rounded(tmp_path):
    exe = str(tmp_path / "tan_cr_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe,
                    os.path.join(ROOT, "tests", "tan_cr_check.cpp"), "-lm"], check=True)
    x = np.ascontiguousarray(_args(20000), dtype="<f8")
    r = subprocess.run([exe], input=x.tobytes(), capture_output=True, check=True)
    got = np.frombuffer(r.stdout, dtype="<f8")
    assert got.shape == x.shape
    want = np.array([cr_tan(v) for v in x])
    bad = np.flatnonzero(got.view(np.int64) != want.view(np.int64))
    assert bad.size == 0, [(repr(x[i]), repr(got[i]), repr(want[i])) for i in bad[:5]]
    # glibc (the reference's math.tan) is not correctly rounded everywhere:
    # the reason the flag parity is stated against the correctly rounded tan
    glibc = np.array([math.tan(v) for v in x])
    assert (glibc != want).sum() < 0.01 * x.size
