#!/bin/bash
# A/B of prebuilt libskillshot variants (ab/*.so, built on the CPU side):
# for each, the fused-step sweep and a short bench line.  Stops at the first
# fault / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=${1:-libab}
OUT=gpurun_out/libab_$TAG.jsonl; : > $OUT
for f in ab/*.so; do
  n=$(basename $f .so)
  SK_LIB_PATH=$PWD/$f timeout -k 10 200 python tools/sweep.py --variants 0 --envs ${ENVS:-65536,262144} --steps 2000 \
    > gpurun_out/sw_$n.jsonl 2> gpurun_out/sw_$n.err; rc=$?
  sed "s/^/{\"lib\": \"$n\", \"r\": /; s/$/}/" gpurun_out/sw_$n.jsonl >> $OUT
  [ $rc -ne 0 ] && { tail -3 gpurun_out/sw_$n.err; exit $rc; }
  [ -n "$NOBENCH" ] && continue
  SK_LIB_PATH=$PWD/$f timeout -k 10 300 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline --no-large --no-learner \
    > gpurun_out/bench_$n.json 2> gpurun_out/bench_$n.err; rc=$?
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_$n.json')); print(json.dumps({'lib':'$n','bench_us':d['roofline']['kernel_us'],'value':d['value'],'rollout':d.get('rollout_random',{}).get('env_steps_per_s_per_gpu')}))" >> $OUT
  [ $rc -ne 0 ] && { tail -3 gpurun_out/bench_$n.err; exit $rc; }
done
cat $OUT
