#!/bin/bash
# A/B: learner ticks per captured graph (2, the default, vs 10) for config 3
# fp32 / bf16 and config 5 on one GPU fp32, 3 alternating passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03g2; mkdir -p $O
: > $O/tpg_ab.jsonl
for rep in 1 2 3; do
  for tpg in 2 10; do
    SK_TICKS_PER_GRAPH=$tpg timeout -k 10 200 python -u -c "
import json, bench
for envs, ex, pr in ((4096, 'action_noise', 'fp32'), (4096, 'action_noise', 'bf16'), (65536, 'param_noise', 'fp32'), (65536, 'param_noise', 'bf16')):
    r = bench.learner_rate(envs, 1, 0, 400, batch=256, exploration=ex, precision=pr)
    print(json.dumps(dict(tpg=$tpg, rep=$rep, envs=envs, precision=pr, us_per_tick=round(r['ms_per_tick'] * 1e3, 2), gpu_us=round(r['gpu_ms_per_tick'] * 1e3, 2))), flush=True)
" >> $O/tpg_ab.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
cat $O/tpg_ab.jsonl
