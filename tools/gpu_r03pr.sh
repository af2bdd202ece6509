#!/bin/bash
# the learner tick's stream priority (SK_TICK_PRIORITY 0 / -1: the update /
# graph stream high): config 5 (streams form) and config 3, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03pr; mkdir -p $O
: > $O/ticks.jsonl
for rep in 1 2; do
  for pr in 0 -1; do
    SK_TICK_PRIORITY=$pr timeout -k 10 300 python -u -c "
import json, bench
for envs, ex, p in ((65536, 'param_noise', 'fp32'), (65536, 'param_noise', 'bf16'), (4096, 'action_noise', 'fp32')):
    r = bench.learner_rate(envs, 1, 0, 400, batch=256, exploration=ex, precision=p)
    print(json.dumps(dict(rep=$rep, prio=$pr, envs=envs, precision=p, tick_mode=r['tick_mode'], us_per_tick=round(r['ms_per_tick'] * 1e3, 2))), flush=True)
" >> $O/ticks.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
cat $O/ticks.jsonl
