#!/bin/bash
# the headline (88-B form) at K = 20 / 4,000: workgroup 64 vs 256 lanes and
# the restart draw under the loads, 3 alternating passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03mb2; mkdir -p $O
: > $O/bench.jsonl
F="--no-learner --no-cpu-baseline --no-large --no-full --no-rollout --no-variants"
for rep in 1 2 3; do
  for cfg in "256 0" "64 0" "256 1" "64 1"; do
    set -- $cfg
    for k in 20 4000; do
      SK_MULTI_BLOCK=$1 SK_MULTI_EARLY=$2 timeout -k 10 200 python -u bench.py --steps $k --warmup 5 $F > $O/b.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
      python3 -c "
import json; d = json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print(json.dumps(dict(rep=$rep, block=$1, early=$2, steps=$k, wall_us=round(d['ms_per_step']*1e3, 3), event_us=round(d['config']['event_ms_per_step']*1e3, 3), frac=round(d['roofline']['frac'], 4), dones=d['episodes']['dones'])))" >> $O/bench.jsonl
    done
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r03mb2/bench.jsonl"):
    x = json.loads(l); d[(x["steps"], x["block"], x["early"])].append((x["event_us"], x["wall_us"]))
for k in sorted(d): print(k, "event", [v[0] for v in d[k]], "wall", [v[1] for v in d[k]])
PY
