#!/bin/bash
# learner GPU tests; bf16 packed-epilogue A/B; learner ticks (config 3 / 5 on
# one GPU, both precisions) with the bf16 minibatch drawn in the critic launch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03w2; mkdir -p $O
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 400 python -u -m pytest tests/test_critic_gpu.py tests/test_actor_gpu.py tests/test_update_gpu.py tests/test_replay_gpu.py tests/test_config3_gpu.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; grep -E "^(FAILED|ERROR)" $O/pytest.txt; tail -2 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_r03y4.sh | grep -v '"param_noise": 0.0' || exit 1
: > $O/ticks.jsonl
for rep in 1 2; do
  timeout -k 10 200 python -u -c "
import json, bench
for envs, ex, pr in ((4096, 'action_noise', 'fp32'), (4096, 'action_noise', 'bf16'), (65536, 'param_noise', 'fp32'), (65536, 'param_noise', 'bf16')):
    r = bench.learner_rate(envs, 1, 0, 400, batch=256, exploration=ex, precision=pr)
    print(json.dumps(dict(rep=$rep, envs=envs, precision=pr, us_per_tick=round(r['ms_per_tick'] * 1e3, 2))), flush=True)
" >> $O/ticks.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
done
cat $O/ticks.jsonl
