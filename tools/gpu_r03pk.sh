#!/bin/bash
# packed resident form (SK_MULTI_PACK) against the 88-B form per launch
# length: the headline at K = 20 (one 20-tick launch), 100, 4,000, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03pk; mkdir -p $O
: > $O/bench.jsonl
F="--no-learner --no-cpu-baseline --no-large --no-full --no-rollout --no-variants"
for rep in 1 2 3; do
  for pk in 1 0; do
    for k in 20 100 4000; do
      SK_MULTI_PACK=$pk timeout -k 10 200 python -u bench.py --steps $k --warmup 5 $F > $O/b.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
      python3 -c "
import json; d = json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print(json.dumps(dict(rep=$rep, pack=$pk, steps=$k, value=d['value'], wall_us=round(d['ms_per_step']*1e3, 3), event_us=round(d['config']['event_ms_per_step']*1e3, 3), frac=round(d['roofline']['frac'], 4), dones=d['episodes']['dones'])))" >> $O/bench.jsonl
    done
  done
done
cat $O/bench.jsonl
