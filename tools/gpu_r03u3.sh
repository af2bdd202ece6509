#!/bin/bash
# A/B: fp32 actor tile with the observations loaded first and then every
# weight operand preloaded, at <= one tile per CU (default) vs per-phase loads
# (SK_FWD_PRE=0): actor forward at 2,048 / 8,192 rows and the config-3 fp32
# learner tick, 3 alternating passes; the act+step trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03u3; mkdir -p $O
: > $O/fwd_ab.jsonl; : > $O/tick_ab.jsonl
for rep in 1 2 3; do
  for v in 0 1; do
    SK_FWD_PRE=$v SK_FWD16=0 timeout -k 10 120 python -u tools/bench_actor_fwd.py --precisions fp32 --rows 2048,8192 2> $O/err.txt | sed "s/^{/{\"fwd_pre\": $v, \"rep\": $rep, /" >> $O/fwd_ab.jsonl || { tail -20 $O/err.txt; exit 1; }
    SK_FWD_PRE=$v timeout -k 10 120 python -u -c "
import json, bench
r = bench.learner_rate(4096, 1, 0, 400, batch=256, exploration='action_noise', precision='fp32')
print(json.dumps(dict(fwd_pre=$v, rep=$rep, us_per_tick=round(r['ms_per_tick'] * 1e3, 2))))" >> $O/tick_ab.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
cat $O/fwd_ab.jsonl $O/tick_ab.jsonl
SK_LIB_PATH=$PWD/ab/trace32.so timeout -k 10 120 python -u tools/trace_act_step.py --noise action --games 4096 > $O/trace_act_step.jsonl 2>&1; tail -1 $O/trace_act_step.jsonl
