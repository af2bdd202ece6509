"""Host check of the step kernels' trig (csrc/sk_trig.hpp), compiled for the
CPU with the kernels' flags: sincos_bf within 1 ulp of glibc (the reference's
math.sin/cos), sincos_fast within SKT_FAST_ERR/2 of long-double sinl/cosl —
the bound the fp32 fast tick's exact-fallback threshold is derived from."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_trig_error_bounds(tmp_path):
    exe = str(tmp_path / "trig_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe,
                    os.path.join(ROOT, "tests", "trig_check.cpp"), "-lm"], check=True)
    r = subprocess.run([exe, "2000000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    fields = dict(kv.split("=") for kv in r.stdout.split())
    assert int(fields["max_ulp_bf"]) <= 1
    assert float(fields["max_err_fast"]) <= 1.5e-7
    assert float(fields["max_err_add"]) <= 3.0e-7
