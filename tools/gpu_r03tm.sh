#!/bin/bash
# per-wave timeline of k_step_multi (trace build): the short launch's fixed cost
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03tm; mkdir -p $O
: > $O/trace.jsonl
for cfg in "65536 20" "65536 100" "8192 20"; do
  set -- $cfg
  SK_LIB_PATH=$PWD/ab/trace_multi.so timeout -k 10 120 python -u tools/trace_multi.py --envs $1 --ticks $2 >> $O/trace.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
done
cat $O/trace.jsonl
