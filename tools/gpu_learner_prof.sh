#!/bin/bash
# rocprofv3 kernel stats of the learner tick (bench.learner_rate) per config and
# precision: bash tools/gpu_learner_prof.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
T=${1:-lp}; O=gpurun_out/$T; mkdir -p $O
for cfg in "4096 action_noise fp32" "4096 action_noise bf16" "65536 param_noise fp32" "65536 param_noise bf16"; do
  set -- $cfg; n=$1; ex=$2; pr=$3; tag=${n}_${pr}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 -c "
import bench, json
r = bench.learner_rate($n, 1, 0, 200, batch=256, exploration='$ex', precision='$pr')
print(json.dumps(r))" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  find $O/$tag -name "*kernel_stats.csv" -exec cp {} $O/stats_$tag.csv \;
  echo "== $tag $(python3 -c "import json; d=json.load(open('$O/$tag.json')); print(round(d['ms_per_tick']*1e3,1), 'us/tick')")"
  python3 - "$O/stats_$tag.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f'{int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:8.2f} us  {r["Name"][:90]}')
PY
done
