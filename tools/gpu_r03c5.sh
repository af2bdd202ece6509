#!/bin/bash
# config 5 on one GPU (fp32, parameter noise): the overlapped tick's forms
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03c5; mkdir -p $O
: > $O/ticks.jsonl
for rep in 1 2; do
  for ov in 1 fused 0; do
    SK_TICK_OVERLAP=$ov timeout -k 10 200 python -u -c "
import json, bench
for envs, pr in ((65536, 'fp32'), (16384, 'fp32')):
    r = bench.learner_rate(envs, 1, 0, 200, batch=256, exploration='param_noise', precision=pr)
    print(json.dumps(dict(rep=$rep, overlap='$ov', envs=envs, precision=pr, tick_mode=r['tick_mode'], us_per_tick=round(r['ms_per_tick'] * 1e3, 2))), flush=True)
" >> $O/ticks.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
cat $O/ticks.jsonl
