#!/bin/bash
# Alternating bench A/B of prebuilt libskillshot variants (ab/*.so, built on
# the CPU side): three passes over the libraries, one bench line each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
for r in 1 2 3; do for f in ab/*.so; do n=$(basename $f .so)
  SK_LIB_PATH=$PWD/$f timeout -k 10 200 python bench.py --steps 4000 --warmup 400 --no-cpu-baseline --no-large --no-learner --no-rollout > gpurun_out/b_${n}_${r}.json 2>gpurun_out/b_err.txt || exit 3
  python -c "import json; d=json.load(open('gpurun_out/b_${n}_${r}.json')); print(json.dumps({'lib':'$n','round':$r,'bench_us':d['roofline']['kernel_us'],'value':d['value']}))" | tee -a gpurun_out/ab_bench.jsonl
done; done
