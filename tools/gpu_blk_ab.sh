#!/bin/bash
# Step-kernel workgroup size A/B: ab/blk*.so (built with -DSK_STEP_BLOCK=…),
# every fused-step variant x batch size, step-only and with obs/reward.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=${1:-blk}
OUT=gpurun_out/blkab_$TAG.jsonl; : > $OUT
for pass in 1 2; do
for f in ab/blk*.so; do
  n=$(basename $f .so)
  for obs in "" "--obs"; do
    SK_LIB_PATH=$PWD/$f timeout -k 10 200 python tools/sweep.py --variants ${VARIANTS:-0,1,2} --envs ${ENVS:-65536,262144,1048576} \
      --steps 2000 $obs > gpurun_out/sw_$n.jsonl 2> gpurun_out/sw_$n.err; rc=$?
    sed "s/^/{\"lib\": \"$n\", \"pass\": $pass, \"r\": /; s/$/}/" gpurun_out/sw_$n.jsonl >> $OUT
    [ $rc -ne 0 ] && { tail -3 gpurun_out/sw_$n.err; exit $rc; }
  done
done
done
echo done
