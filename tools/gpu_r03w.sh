#!/bin/bash
# round-3 re-entry check: full GPU test suite, then rocprof kernel stats of the
# config-3 learner tick (fp32 + bf16)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -3 $O/pytest_gpu.txt
for pr in fp32 bf16; do
  tag=4096_$pr
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 -c "
import bench, json
r = bench.learner_rate(4096, 1, 0, 200, batch=256, exploration='action_noise', precision='$pr')
print(json.dumps(r))" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  find $O/$tag -name "*kernel_stats.csv" -exec cp {} $O/stats_$tag.csv \;
  echo "== $tag $(python3 -c "import json; d=json.load(open('$O/$tag.json')); print(round(d['ms_per_tick']*1e3,1), 'us/tick')")"
  python3 - "$O/stats_$tag.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:8.2f} us  {r["Name"][:100]}')
PY
done
