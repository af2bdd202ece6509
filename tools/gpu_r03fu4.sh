#!/bin/bash
# the whole GPU suite and smoke on the fused / overlapped ticks, then learner
# ticks in the default (auto) mode: config 3 and config 5 on one GPU, both
# precisions
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03fu4; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; grep -E "^(FAILED|ERROR)" $O/pytest.txt; tail -2 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -3 $O/smoke.txt
: > $O/ticks.jsonl
for rep in 1 2; do
  timeout -k 10 300 python -u -c "
import json, bench
for envs, ex, pr in ((4096, 'action_noise', 'fp32'), (4096, 'action_noise', 'bf16'), (65536, 'param_noise', 'fp32'), (65536, 'param_noise', 'bf16')):
    r = bench.learner_rate(envs, 1, 0, 400, batch=256, exploration=ex, precision=pr)
    print(json.dumps(dict(rep=$rep, envs=envs, precision=pr, tick_mode=r['tick_mode'], us_per_tick=round(r['ms_per_tick'] * 1e3, 2), gpu_us=round(r['gpu_ms_per_tick'] * 1e3, 2))), flush=True)
" >> $O/ticks.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
done
cat $O/ticks.jsonl
