#!/bin/bash
# the multi-tick tests on the 256-lane default; trace of the first tick with
# and without the packed resident form
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03mc; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_multi_gpu.py tests/test_bench_path_gpu.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; grep -E "^(FAILED|ERROR)" $O/pytest.txt; tail -2 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
: > $O/trace.jsonl
for pk in 1 0; do
  SK_MULTI_PACK=$pk SK_LIB_PATH=$PWD/ab/trace_multi.so timeout -k 10 120 python -u tools/trace_multi.py --envs 65536 --ticks 20 | sed "s/^{/{\"pack\": $pk, /" >> $O/trace.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
done
cat $O/trace.jsonl | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); x = d['launches'][-1]
    print(d['pack'], 'entry_spread', x['entry_spread_us'], 'ticks', x['tick_p50_us'][:4], x['tick_p50_us'][-3:], 'last->exit', x['last_tick_to_exit_p50_us'], 'span', x['span_us'])"
