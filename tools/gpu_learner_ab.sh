#!/bin/bash
# Learner-in-the-loop throughput, fused (MFMA) update vs the autograd path,
# graph-replayed ticks (tools/bench_learner.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=${1:-lab}
OUT=gpurun_out/learner_$TAG.jsonl; : > $OUT
for cfg in "4096 256" "4096 4096" "65536 4096"; do
  set -- $cfg
  for fused in 1 0; do
    SK_FUSED_UPDATE=$fused timeout -k 10 240 python tools/bench_learner.py --envs $1 --batch $2 --graph --ticks 200 \
      > gpurun_out/lb.json 2> gpurun_out/lb.err; rc=$?
    [ $rc -ne 0 ] && { tail -5 gpurun_out/lb.err; exit $rc; }
    python -c "import json; d=json.load(open('gpurun_out/lb.json')); d['fused_update']=$fused; print(json.dumps(d))" >> $OUT
  done
done
cat $OUT
