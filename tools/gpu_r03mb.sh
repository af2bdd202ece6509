#!/bin/bash
# k_step_multi: DPP counter reduction (trace), and 64- vs 256-lane workgroups
# (SK_MULTI_BLOCK) on the headline at K = 20 (driver) and K = 4,000, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03mb; mkdir -p $O
: > $O/trace.jsonl
for mb in 64 256; do
  SK_MULTI_BLOCK=$mb SK_LIB_PATH=$PWD/ab/trace_multi.so timeout -k 10 120 python -u tools/trace_multi.py --envs 65536 --ticks 20 | sed "s/^{/{\"block\": $mb, /" >> $O/trace.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
done
: > $O/bench.jsonl
F="--no-learner --no-cpu-baseline --no-large --no-full --no-rollout --no-variants"
for rep in 1 2 3; do
  for mb in 64 256; do
    for k in 20 4000; do
      SK_MULTI_BLOCK=$mb timeout -k 10 200 python -u bench.py --steps $k --warmup 5 $F > $O/b.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
      python3 -c "
import json; d = json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print(json.dumps(dict(rep=$rep, block=$mb, steps=$k, value=d['value'], wall_us=round(d['ms_per_step']*1e3, 3), event_us=round(d['config']['event_ms_per_step']*1e3, 3), frac=round(d['roofline']['frac'], 4), episodes=d.get('episodes'))))" >> $O/bench.jsonl
    done
  done
done
cat $O/trace.jsonl | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); x = d['launches'][-1]
    print(d['block'], 'entry_spread', x['entry_spread_us'], 'tick0', x['tick_p50_us'][0], 'tick5', x['tick_p50_us'][5], 'last->exit', x['last_tick_to_exit_p50_us'], 'span', x['span_us'])"
cat $O/bench.jsonl
