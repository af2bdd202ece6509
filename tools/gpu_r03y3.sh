#!/bin/bash
# A/B: bf16 noisy actor forward: normals16 + noisy_pre (ab/noise_base.so) vs
# the Box-Muller pair form with one sqrt per element (current, Philox 10
# rounds) vs the pair form at Philox4x32-7 (ab/noise_pair7.so), 3
# alternating passes; then the distribution test on the current build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03y3; mkdir -p $O
: > $O/noise_ab.jsonl
for rep in 1 2 3; do
  for v in base pair10 pair7; do
    case $v in base) export SK_LIB_PATH=$PWD/ab/noise_base.so;; pair7) export SK_LIB_PATH=$PWD/ab/noise_pair7.so;; *) unset SK_LIB_PATH;; esac
    timeout -k 10 120 python -u tools/bench_actor_fwd.py --precisions bf16 --rows 8192,131072 2> $O/err.txt | grep '"param_noise": 0.5' | sed "s/^{/{\"variant\": \"$v\", \"rep\": $rep, /" >> $O/noise_ab.jsonl || { tail -20 $O/err.txt; exit 1; }
  done
done
unset SK_LIB_PATH
cat $O/noise_ab.jsonl
timeout -k 10 200 python -u -m pytest tests/test_actor_gpu.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_actor.txt 2>&1; tail -3 $O/pytest_actor.txt
