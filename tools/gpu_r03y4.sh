#!/bin/bash
# A/B: bf16 actor forward with the pair-form epilogues in packed fp32 (current)
# vs scalar (ab/unpacked.so), 3 alternating passes, noise on/off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03y4; mkdir -p $O
: > $O/actor_ab.jsonl
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export SK_LIB_PATH=$PWD/ab/unpacked.so; else unset SK_LIB_PATH; fi
    timeout -k 10 120 python -u tools/bench_actor_fwd.py --precisions bf16 --rows 8192,131072 2> $O/err.txt | sed "s/^{/{\"variant\": \"$v\", \"rep\": $rep, /" >> $O/actor_ab.jsonl || { tail -20 $O/err.txt; exit 1; }
  done
done
cat $O/actor_ab.jsonl
