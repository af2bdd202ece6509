#!/bin/bash
# the acting launch on 16-row tiles (k_act_step16, SK_ACT16): parity tests,
# then config-3 fp32 ticks (fused and sequential) with SK_ACT16=0 / 1, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03a16; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_replay_gpu.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; grep -E "^(FAILED|ERROR)" $O/pytest.txt; tail -2 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
: > $O/ticks.jsonl
for rep in 1 2 3; do
  for a16 in 0 1; do
    SK_ACT16=$a16 timeout -k 10 300 python -u -c "
import json, os, bench
for ov, envs, ex in (('auto', 4096, 'action_noise'), ('auto', 4096, 'param_noise'), ('0', 4096, 'action_noise'), ('auto', 8192, 'param_noise')):
    os.environ['SK_TICK_OVERLAP'] = ov
    r = bench.learner_rate(envs, 1, 0, 400, batch=256, exploration=ex, precision='fp32')
    print(json.dumps(dict(rep=$rep, act16=$a16, envs=envs, exploration=ex, tick_mode=r['tick_mode'], us_per_tick=round(r['ms_per_tick'] * 1e3, 2))), flush=True)
" >> $O/ticks.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
cat $O/ticks.jsonl
