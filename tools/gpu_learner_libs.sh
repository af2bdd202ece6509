#!/bin/bash
# A/B of prebuilt library variants (ab/*.so) on the learner-in-the-loop tick
# (tools/bench_learner.py, hipGraph) and the critic/actor update kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
for f in ab/*.so; do
  n=$(basename $f .so)
  for e in ${ENVS:-4096}; do
    SK_LIB_PATH=$PWD/$f timeout -k 10 120 python tools/bench_learner.py --graph --envs $e --ticks 400 \
      | sed "s/^{/{\"lib\": \"$n\", /" || exit $?
  done
  SK_LIB_PATH=$PWD/$f timeout -k 10 120 python tools/bench_mlp_kernels.py --rows 4096 --only ${ONLY:-critic_grad_boot} \
    | sed "s/^{/{\"lib\": \"$n\", /" || exit $?
done
