"""Build libskillshot.so (the HIP engine + C ABI) in-tree for gfx950.

    python -m skillshot_learning_amd.build

Cross-compiles without a GPU.  The .so lands in skillshot_learning_amd/lib/
(git-ignored, but it travels to the GPU box with the gpurun snapshot).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_DIR = os.path.join(HERE, "lib")
# SK_LIB_PATH: load a prebuilt variant instead (A/B experiments, tools/gpu_lib_ab.sh)
LIB_PATH = os.environ.get("SK_LIB_PATH") or os.path.join(LIB_DIR, "libskillshot.so")
# csrc/sk_diag.hip (measurement-only kernels: the copy floor) is not part of
# the product library: tools/build_variant.sh builds it into diagnostic
# variants (tools/sweep.py --diag loads one through SK_LIB_PATH)
SOURCES = [os.path.join(HERE, "csrc", "sk_engine.hip"), os.path.join(HERE, "csrc", "sk_actor.hip"),
           os.path.join(HERE, "csrc", "sk_critic.hip"), os.path.join(HERE, "csrc", "sk_update.hip"),
           os.path.join(HERE, "csrc", "sk_replay.hip"), os.path.join(HERE, "csrc", "sk_learn32.hip"),
           os.path.join(HERE, "csrc", "sk_fit.hip"),
           os.path.join(HERE, "csrc", "sk_host.cpp")]
DEPS = SOURCES + [os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc"))
                  if f.endswith((".hpp", ".h", ".cpp"))] + [os.path.join(ROOT, "include", "skillshot.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -ffp-contract=off: the reference's fp64 op order must survive (no FMA
# contraction of x - sin(r)*5); code object v5 loads under both the image's
# ROCm 7.2 runtime and torch's bundled 7.0 runtime.
FLAGS = ["-O3", "--offload-arch=gfx950", "-fPIC", "-shared", "-std=c++17", "-ffp-contract=off",
         "-mcode-object-version=5", "-Wall", "-Werror=return-type"]


def needs_build():
    if os.environ.get("SK_LIB_PATH"):
        return False
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(p) > t for p in DEPS)


def build(force=False, verbose=False):
    if not force and not needs_build():
        return LIB_PATH
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = LIB_PATH + ".tmp"
    cmd = [HIPCC] + FLAGS + ["-I", os.path.join(ROOT, "include"), "-o", tmp] + SOURCES
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
