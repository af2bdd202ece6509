#!/bin/bash
# Alternating A/B of prebuilt library variants (ab_run/*.so, SK_LIB_PATH) on
# the one-tick step kernels and the fused acting launch
# (tools/bench_step_kernels.py):   PASSES=2 bash tools/ab_libs_step.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
OUT=gpurun_out/${1:-ab_libs_step}.jsonl; : > $OUT
for r in $(seq ${PASSES:-2}); do for f in ab_run/*.so; do n=$(basename $f .so)
  SK_LIB_PATH=$PWD/$f timeout -k 10 200 python3 tools/bench_step_kernels.py ${ARGS:-} | sed "s/^{/{\"lib\": \"$n\", \"round\": $r, /" >> $OUT || exit 3
done; done
cat $OUT
