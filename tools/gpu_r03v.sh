#!/bin/bash
# A/B: sliced Adam with the W1 / b1 contribution rows summed by 16 x 16
# workgroups (current) vs 64 x 4 (ab/adam_old.so): the config-3 fp32 learner
# tick, 3 alternating passes; then the update / learner GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03v; mkdir -p $O
: > $O/adam_tick_ab.jsonl
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export SK_LIB_PATH=$PWD/ab/adam_old.so; else unset SK_LIB_PATH; fi
    timeout -k 10 120 python -u -c "
import json, bench
r = bench.learner_rate(4096, 1, 0, 400, batch=256, exploration='action_noise', precision='fp32')
print(json.dumps(dict(variant='$v', rep=$rep, us_per_tick=round(r['ms_per_tick'] * 1e3, 2))))" >> $O/adam_tick_ab.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
unset SK_LIB_PATH
cat $O/adam_tick_ab.jsonl
timeout -k 10 300 python -u -m pytest tests/test_update_gpu.py tests/test_learn32_gpu.py tests/test_config3_gpu.py tests/test_replay_gpu.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; tail -3 $O/pytest.txt
