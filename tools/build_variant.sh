#!/usr/bin/env bash
# Build a libskillshot variant with extra compile flags (A/B experiments,
# diagnostic trace builds):  tools/build_variant.sh OUT.so [-DFLAG ...]
# Load it with SK_LIB_PATH=$PWD/OUT.so.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$1"; shift
SRC=(sk_engine.hip sk_diag.hip sk_actor.hip sk_critic.hip sk_update.hip sk_replay.hip sk_learn32.hip sk_fit.hip sk_host.cpp)
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -shared -std=c++17 -ffp-contract=off -mcode-object-version=5 \
  -Wall -Werror=return-type "$@" -I "$ROOT/include" -o "$OUT" "${SRC[@]/#/$ROOT/skillshot_learning_amd/csrc/}"
