#!/bin/bash
# k_act_step32 codegen A/B (static LDS / dynamic LDS / dynamic + by-value
# args): config-3 fp32 ticks, sequential and fused, alternating libraries
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03fu3; mkdir -p $O
: > $O/ticks.jsonl
for rep in 1 2; do
  for v in a_static b_dynamic c_byval; do
    SK_LIB_PATH=$PWD/ab/$v.so timeout -k 10 200 python -u -c "
import json, os, bench
for ov in ('0', 'fused'):
    os.environ['SK_TICK_OVERLAP'] = ov
    r = bench.learner_rate(4096, 1, 0, 400, batch=256, exploration='action_noise', precision='fp32')
    print(json.dumps(dict(rep=$rep, lib='$v', overlap=ov, us_per_tick=round(r['ms_per_tick'] * 1e3, 2))), flush=True)
" >> $O/ticks.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
cat $O/ticks.jsonl
