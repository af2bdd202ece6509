#!/bin/bash
# A/B sweep of fused-step variants x batch sizes (no tests).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=${1:-ab}
timeout -k 10 400 python tools/sweep.py ${SWEEP_ARGS:-} > gpurun_out/sweep_$TAG.jsonl 2>gpurun_out/sweep_$TAG.err; rc=$?
cat gpurun_out/sweep_$TAG.jsonl; tail -3 gpurun_out/sweep_$TAG.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/sweep.py --obs --envs 65536,1048576 > gpurun_out/sweep_obs_$TAG.jsonl 2>>gpurun_out/sweep_$TAG.err
cat gpurun_out/sweep_obs_$TAG.jsonl
