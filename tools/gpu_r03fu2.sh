#!/bin/bash
# rocprofv3 kernel stats of the config-3 fp32 tick, sequential (SK_TICK_OVERLAP=0)
# and fused (the acting launch in the actor backward's launch)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03fu2; mkdir -p $O
for ov in 0 fused; do
  tag=c3_fp32_ov$ov
  SK_TICK_OVERLAP=$ov timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 -c "
import bench, json
r = bench.learner_rate(4096, 1, 0, 200, batch=256, exploration='action_noise', precision='fp32')
print(json.dumps(r))" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  find $O/$tag -name "*kernel_stats.csv" -exec cp {} $O/stats_$tag.csv \;
  rm -rf $O/$tag
  echo "== $tag $(python3 -c "import json; d=json.load(open('$O/$tag.json')); print(round(d['ms_per_tick']*1e3,1), 'us/tick')")"
  python3 - "$O/stats_$tag.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:8]:
    print(f'{int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:8.2f} us  {r["Name"][:90]}')
PY
done
