#!/bin/bash
# the 88-B multi-tick kernels re-swept at the headline size: restart draw
# under the loads (early), split geometry, workgroup size
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03ms; mkdir -p $O
timeout -k 10 400 python -u tools/multi_sweep.py --envs 65536 --ticks 20,400 --pols 1 --reps 2 --splits 0,1 --earlys 0,1 --blocks=-1,64 --no-graph > $O/sweep.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r03ms/sweep.jsonl"):
    x = json.loads(l)
    if x.get("kind") != "multi": continue
    d[(x["ticks_per_launch"], x["split"], x["early"], x["block"])].append(x["us_per_tick"])
for k in sorted(d): print(k, [round(v, 3) for v in d[k]])
PY
