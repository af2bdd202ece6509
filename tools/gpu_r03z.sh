#!/bin/bash
# A/B of the driver's short region (bench.py --steps 20 --warmup 5, headline
# leg only): HSA signal waits by interrupt (default) vs polling
# (HSA_ENABLE_INTERRUPT=0), 4 alternating passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03z; mkdir -p $O
: > $O/k20_interrupt_ab.jsonl
for rep in 1 2 3 4; do
  for v in 1 0; do
    HSA_ENABLE_INTERRUPT=$v timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-learner --no-cpu-baseline --no-large --no-full --no-rollout --no-variants > $O/b.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
    python3 -c "
import json; d = json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print(json.dumps(dict(rep=$rep, hsa_enable_interrupt=$v, value=d['value'], wall_us=d['ms_per_step']*1e3, event_us=d['config']['event_ms_per_step']*1e3, episodes=d.get('episodes'))))" >> $O/k20_interrupt_ab.jsonl
  done
done
cat $O/k20_interrupt_ab.jsonl
