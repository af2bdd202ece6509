#!/bin/bash
# the acting tick carried by the critic's backward launch vs the actor's:
# parity tests, then config-3 fp32 ticks (SK_FUSE_ACT_IN), alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03fc; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_replay_gpu.py tests/test_config3_gpu.py tests/test_learn32_gpu.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; grep -E "^(FAILED|ERROR)" $O/pytest.txt; tail -2 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
: > $O/ticks.jsonl
for rep in 1 2 3; do
  for c in critic actor; do
    SK_FUSE_ACT_IN=$c timeout -k 10 200 python -u -c "
import json, bench
for ex in ('action_noise', 'param_noise'):
    r = bench.learner_rate(4096, 1, 0, 400, batch=256, exploration=ex, precision='fp32')
    print(json.dumps(dict(rep=$rep, carrier='$c', exploration=ex, tick_mode=r['tick_mode'], us_per_tick=round(r['ms_per_tick'] * 1e3, 2))), flush=True)
" >> $O/ticks.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
cat $O/ticks.jsonl
