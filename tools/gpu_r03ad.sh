#!/bin/bash
# k_adam_flat partial-read slices (SK_ADAM_SLICES 4 / 8 / 16 waves per 64
# parameters): learner ticks, config 3 (fp32, bf16) and config 5 fp32 on one
# GPU, alternating library variants ab/adam*.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03ad; mkdir -p $O
: > $O/ticks.jsonl
for rep in 1 2; do
  for v in adam4 adam8 adam16; do
    SK_LIB_PATH=$PWD/ab/$v.so timeout -k 10 200 python -u -c "
import json, bench
for envs, ex, pr in ((4096, 'action_noise', 'fp32'), (4096, 'action_noise', 'bf16'), (65536, 'param_noise', 'fp32')):
    r = bench.learner_rate(envs, 1, 0, 400, batch=256, exploration=ex, precision=pr)
    print(json.dumps(dict(rep=$rep, lib='$v', envs=envs, precision=pr, us_per_tick=round(r['ms_per_tick'] * 1e3, 2))), flush=True)
" >> $O/ticks.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
cat $O/ticks.jsonl
