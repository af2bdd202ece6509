#!/bin/bash
# learner ticks per captured graph (SK_TICKS_PER_GRAPH 2 / 10 / 20) on the
# current ticks: config 3 fp32 (fused) and bf16, config 5 fp32 (streams), alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03tpg; mkdir -p $O
: > $O/ticks.jsonl
for rep in 1 2; do
  for tpg in 2 10 20; do
    SK_TICKS_PER_GRAPH=$tpg timeout -k 10 300 python -u -c "
import json, bench
for envs, ex, pr in ((4096, 'action_noise', 'fp32'), (4096, 'action_noise', 'bf16'), (65536, 'param_noise', 'fp32')):
    r = bench.learner_rate(envs, 1, 0, 400, batch=256, exploration=ex, precision=pr)
    print(json.dumps(dict(rep=$rep, tpg=$tpg, envs=envs, precision=pr, tick_mode=r['tick_mode'], us_per_tick=round(r['ms_per_tick'] * 1e3, 2), gpu_us=round(r['gpu_ms_per_tick'] * 1e3, 2))), flush=True)
" >> $O/ticks.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
cat $O/ticks.jsonl
