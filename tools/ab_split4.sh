#!/bin/bash
# Timing ablation of the split multi-tick kernel's trig:
# ab_run/split_{base,noqsc,nosc}.so built by tools/build_variant.sh with no
# flag, -DSK_ABL_NOQSC (no projectile sincos) and -DSK_ABL_NOSC (no sincos):
# µs per tick at ENVS games, 400 ticks per launch, write-through port, two
# lanes per game, the action-slab prefetch wave.  Results are wrong by
# construction in the ablated builds; only their time is read.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
OUT=gpurun_out/${1:-ab_split4}.jsonl; : > $OUT
for rep in 0 1; do
  for n in ${LIBS:-split_base split_noqsc split_nosc}; do
    SK_LIB_PATH=$PWD/ab_run/$n.so timeout -k 10 120 python tools/multi_sweep.py --envs ${ENVS:-8192,16384,32768} \
      --ticks 400 --pols 1 --splits ${SPLITS:-1} --prefetches ${PF:-1} --no-graph --reps 1 > gpurun_out/ab_$n.jsonl || exit $?
    sed "s/^/{\"lib\": \"$n\", \"rep\": $rep, \"r\": /; s/$/}/" gpurun_out/ab_$n.jsonl >> $OUT
  done
done
cat $OUT
