#!/bin/bash
# full GPU suite; config-3 learner tick A/B of the replay fusion modes
# (SK_FUSED_REPLAY 2 = insert in the step, gather in the critic, with the fp32
# actor in the step launch (SK_FUSED_ACT=1) or not; 1 = one insert+sample
# launch), 3 alternating passes; rocprof stats of the default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03x; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu --maxfail=10 -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.txt; tail -3 $O/pytest_gpu.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc  # a fault / abort / timeout ends the call
timeout -k 10 300 python -u - > $O/replay_modes_ab.jsonl 2> $O/replay_modes_ab.err <<'PY' || { tail -20 $O/replay_modes_ab.err; exit 1; }
import json, os, sys
sys.path.insert(0, ".")
import bench
for rep in range(3):
    for mode, act in (("1", "1"), ("2", "0"), ("2", "1")):
        for pr in ("fp32", "bf16"):
            if pr == "bf16" and act == "0":
                continue
            os.environ["SK_FUSED_REPLAY"] = mode
            os.environ["SK_FUSED_ACT"] = act
            r = bench.learner_rate(4096, 1, 0, 400, batch=256, exploration="action_noise", precision=pr)
            print(json.dumps(dict(rep=rep, mode=mode, act=act, precision=pr, us_per_tick=round(r["ms_per_tick"] * 1e3, 2),
                                  gpu_us=round(r["gpu_ms_per_tick"] * 1e3, 2))), flush=True)
PY
cat $O/replay_modes_ab.jsonl
for pr in fp32; do
  tag=4096_$pr
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 -c "
import bench, json
r = bench.learner_rate(4096, 1, 0, 200, batch=256, exploration='action_noise', precision='$pr')
print(json.dumps(r))" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  find $O/$tag -name "*kernel_stats.csv" -exec cp {} $O/stats_$tag.csv \;
  python3 - "$O/stats_$tag.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:8.2f} us  {r["Name"][:100]}')
PY
done
