#!/usr/bin/env bash
# Build libskillshot from the csrc/ + include/ of a git revision (A/B against
# an earlier kernel): tools/build_rev.sh REV OUT.so [-DFLAG ...]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
REV="$1"; OUT="$2"; shift 2
T=$(mktemp -d)
git -C "$ROOT" archive "$REV" skillshot_learning_amd/csrc include | tar -x -C "$T"
SRC=(sk_engine.hip sk_diag.hip sk_actor.hip sk_critic.hip sk_update.hip sk_replay.hip sk_learn32.hip sk_fit.hip sk_host.cpp)
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -shared -std=c++17 -ffp-contract=off -mcode-object-version=5 \
  -Wall -Werror=return-type "$@" -I "$T/include" -o "$OUT" "${SRC[@]/#/$T/skillshot_learning_amd/csrc/}"
rm -rf "$T"
