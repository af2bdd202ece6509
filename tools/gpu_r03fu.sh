#!/bin/bash
# the fused overlapped tick (acting launch in the actor backward's launch):
# parity tests, then config-3 ticks SK_TICK_OVERLAP=0 / fused / auto,
# fp32 action and parameter noise, bf16 and config 5 unchanged, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03fu; mkdir -p $O
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 500 python -u -m pytest tests/test_replay_gpu.py tests/test_config3_gpu.py tests/test_learn32_gpu.py tests/test_update_gpu.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; grep -E "^(FAILED|ERROR)" $O/pytest.txt; tail -2 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
: > $O/ticks.jsonl
for rep in 1 2 3; do
  for ov in 0 fused; do
    SK_TICK_OVERLAP=$ov timeout -k 10 200 python -u -c "
import json, bench
for envs, ex, pr in ((4096, 'action_noise', 'fp32'), (4096, 'param_noise', 'fp32')):
    r = bench.learner_rate(envs, 1, 0, 400, batch=256, exploration=ex, precision=pr)
    print(json.dumps(dict(rep=$rep, overlap='$ov', envs=envs, exploration=ex, precision=pr, us_per_tick=round(r['ms_per_tick'] * 1e3, 2), tick_mode=r['tick_mode'])), flush=True)
" >> $O/ticks.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
cat $O/ticks.jsonl
