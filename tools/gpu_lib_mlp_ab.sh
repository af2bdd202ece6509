#!/bin/bash
# A/B of prebuilt libskillshot variants (ab/*.so) on the MLP kernels
# (tools/bench_mlp_kernels.py), one JSON line per (lib, kernel, rows).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=${1:-mlpab}
OUT=gpurun_out/mlpab_$TAG.jsonl; : > $OUT
for f in ab/*.so; do
  n=$(basename $f .so)
  SK_LIB_PATH=$PWD/$f timeout -k 10 200 python tools/bench_mlp_kernels.py --rows ${ROWS:-8192,131072} ${ONLY:+--only $ONLY} \
    > gpurun_out/mlp_$n.jsonl 2> gpurun_out/mlp_$n.err; rc=$?
  sed "s/^{/{\"lib\": \"$n\", /" gpurun_out/mlp_$n.jsonl >> $OUT
  [ $rc -ne 0 ] && { tail -3 gpurun_out/mlp_$n.err; exit $rc; }
done
cat $OUT
