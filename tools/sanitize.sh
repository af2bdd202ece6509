#!/usr/bin/env bash
# AddressSanitizer + UndefinedBehaviorSanitizer run of the host code (SURVEY.md
# §5): libskillshot with its host code instrumented (the CPU backend
# csrc/sk_host.cpp and the ABI layer; GPU code is not instrumented, and no GPU
# is used) and the C oracle, then the CPU test suites that drive them, with
# the clang ASan runtime preloaded into Python.  CPU only: never on the GPU box.
#   tools/sanitize.sh [pytest args]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/build/asan"
mkdir -p "$OUT"
SAN=(-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined
     -Xarch_host -fno-omit-frame-pointer)
SRC=(sk_engine.hip sk_diag.hip sk_actor.hip sk_critic.hip sk_update.hip sk_replay.hip sk_learn32.hip sk_host.cpp)
/opt/rocm/bin/hipcc -O1 -g --offload-arch=gfx950 -fPIC -shared -std=c++17 -ffp-contract=off -mcode-object-version=5 \
  "${SAN[@]}" -I "$ROOT/include" -o "$OUT/libskillshot.so" "${SRC[@]/#/$ROOT/skillshot_learning_amd/csrc/}"
/opt/rocm/llvm/bin/clang -O1 -g -fPIC -shared -std=c11 -ffp-contract=off -fno-fast-math \
  -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer \
  -o "$OUT/libskillshot_oracle.so" "$ROOT/oracle/skillshot_oracle.c" -lm
RT="$(ls /opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)"
cd "$ROOT"
LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  SK_LIB_PATH="$OUT/libskillshot.so" SK_ORACLE_LIB="$OUT/libskillshot_oracle.so" \
  python -m pytest -q -p no:cacheprovider -m "not gpu" \
  tests/test_host_backend_cpu.py tests/test_game_api.py tests/test_oracle_golden.py tests/test_closed_forms_cpu.py \
  tests/test_capi_cpu.py "$@"
