#!/bin/bash
# k_adam_flat parameters per workgroup (SK_ADAM_PARAMS 16 / 32 / 64 / 128):
# the Adam tests per variant, then config-3 ticks (fp32 fused, bf16), alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03adp; mkdir -p $O
for v in adp16 adp32 adp64 adp128; do
  SK_LIB_PATH=$PWD/ab/$v.so timeout -k 10 300 python -u -m pytest tests/test_update_gpu.py tests/test_learn32_gpu.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_$v.txt 2>&1
  rc=$?; echo "$v $(tail -1 $O/pytest_$v.txt)"; [ $rc -eq 0 ] || exit $rc
done
: > $O/ticks.jsonl
for rep in 1 2; do
  for v in adp64 adp16 adp32 adp128; do
    SK_LIB_PATH=$PWD/ab/$v.so timeout -k 10 200 python -u -c "
import json, bench
for pr in ('fp32', 'bf16'):
    r = bench.learner_rate(4096, 1, 0, 400, batch=256, exploration='action_noise', precision=pr)
    print(json.dumps(dict(rep=$rep, lib='$v', precision=pr, us_per_tick=round(r['ms_per_tick'] * 1e3, 2))), flush=True)
" >> $O/ticks.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
cat $O/ticks.jsonl
