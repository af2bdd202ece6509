#!/bin/bash
# the overlapped learner tick: its GPU tests (graph == eager, exclusion
# sampling) with the learner suites, then SK_TICK_OVERLAP=0 vs 1 on config 3
# and config 5 (one GPU), both precisions, alternating passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03ov; mkdir -p $O
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 500 python -u -m pytest tests/test_replay_gpu.py tests/test_config3_gpu.py tests/test_learn32_gpu.py tests/test_update_gpu.py tests/test_actor_gpu.py tests/test_rccl_capture_gpu.py tests/test_multirank_gpu.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; grep -E "^(FAILED|ERROR)" $O/pytest.txt; tail -2 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
: > $O/ticks.jsonl
for rep in 1 2 3; do
  for ov in 0 1; do
    SK_TICK_OVERLAP=$ov timeout -k 10 200 python -u -c "
import json, bench
for envs, ex, pr in ((4096, 'action_noise', 'fp32'), (4096, 'action_noise', 'bf16'), (65536, 'param_noise', 'fp32'), (65536, 'param_noise', 'bf16')):
    r = bench.learner_rate(envs, 1, 0, 400, batch=256, exploration=ex, precision=pr)
    print(json.dumps(dict(rep=$rep, overlap=$ov, envs=envs, precision=pr, us_per_tick=round(r['ms_per_tick'] * 1e3, 2))), flush=True)
" >> $O/ticks.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
cat $O/ticks.jsonl
