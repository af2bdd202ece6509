#!/bin/bash
# the overlap tests (serial == overlapped), then kernel-trace timelines of the
# config-3 fp32 learner tick with SK_TICK_OVERLAP=0 / 1 (does the acting launch
# run beside the update chain inside the graph?)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03ov2; mkdir -p $O
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 200 python -u -m pytest tests/test_replay_gpu.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "overlap or modes_equal" > $O/pytest.txt 2>&1
rc=$?; grep -E "^(FAILED|ERROR)" $O/pytest.txt; tail -2 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for ov in 0 1; do
 for cfg in "4096 action_noise fp32" "65536 param_noise bf16"; do
  set -- $cfg; n=$1; ex=$2; pr=$3; tag=ov${ov}_${n}_${pr}
  SK_TICK_OVERLAP=$ov timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o run -- python3 -c "
import bench, json
r = bench.learner_rate($n, 1, 0, 100, batch=256, exploration='$ex', precision='$pr')
print(json.dumps(r))" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  f=$(find $O/$tag -name "*kernel_trace.csv" | head -1)
  echo "== $tag"; python3 tools/overlap_timeline.py $f 16 | tee $O/$tag.timeline.txt
  rm -rf $O/$tag
 done
done
