#!/bin/bash
# Alternating A/B (3 passes) of prebuilt ab/*.so on the full-contract tick
# (obs + reward written; k_step_split = variant 1, k_step = variant 0) plus
# the diag floors (empty, copy, copy_full) at ENVS games.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-ab_split}.jsonl; : > $OUT
E=${ENVS:-65536}
for r in 1 2 3; do
  for f in ab/*.so; do n=$(basename $f .so)
    SK_LIB_PATH=$PWD/$f timeout -k 10 200 python tools/sweep.py --variants ${VARIANTS:-1,0} --envs $E ${OBSFLAG---obs} --steps 2000 \
      > /tmp/sw.jsonl 2> /tmp/sw_err.txt || { tail -5 /tmp/sw_err.txt; exit 3; }
    sed "s/^/{\"lib\": \"$n\", \"round\": $r, \"r\": /; s/$/}/" /tmp/sw.jsonl | tee -a $OUT
  done
  timeout -k 10 200 python tools/sweep.py --variants empty,copy,copy_full --envs $E --steps 2000 > /tmp/sw.jsonl 2> /tmp/sw_err.txt || { tail -5 /tmp/sw_err.txt; exit 3; }
  sed "s/^/{\"lib\": \"floor\", \"round\": $r, \"r\": /; s/$/}/" /tmp/sw.jsonl | tee -a $OUT
done
