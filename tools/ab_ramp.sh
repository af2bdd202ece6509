#!/bin/bash
# Alternating A/B (SK_BENCH_RAMP=0 / 1, 4 passes) of the driver-style short
# headline run (bench.py --steps 20 --warmup 5, headline leg only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
OUT=gpurun_out/ab_ramp.jsonl; : > $OUT
for r in 1 2 3 4; do for ramp in 0 1; do
  SK_BENCH_RAMP=$ramp timeout -k 10 200 python bench.py --steps ${K:-20} --warmup 5 --no-cpu-baseline --no-large \
    --no-learner --no-full --no-rollout > /tmp/b.json 2> /tmp/b.err || { tail -5 /tmp/b.err; exit 3; }
  python3 -c "
import json; d = json.load(open('/tmp/b.json'))
print(json.dumps(dict(ramp=$ramp, round=$r, value=d['value'], ms_per_step=d['ms_per_step'], event=d['config']['event_ms_per_step'])))" | tee -a $OUT
done; done
