#!/bin/bash
# Alternating A/B of prebuilt libskillshot variants (ab/*.so) on the learner
# tick's step (k_step_split with obs/reward): tools/sweep.py --obs, 3 passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
for r in 1 2 3; do for f in ab/*.so; do n=$(basename $f .so)
  SK_LIB_PATH=$PWD/$f timeout -k 10 200 python tools/sweep.py --variants 1 --envs ${ENVS:-4096,65536} --obs --steps 2000 \
    > gpurun_out/sw_${n}_${r}.jsonl 2> gpurun_out/sw_err.txt || exit 3
  sed "s/^/{\"lib\": \"$n\", \"round\": $r, \"r\": /; s/$/}/" gpurun_out/sw_${n}_${r}.jsonl | tee -a gpurun_out/ab_sweep_obs.jsonl
done; done
