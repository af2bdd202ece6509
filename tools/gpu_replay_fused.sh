#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/rf
timeout -k 10 600 python -u -m pytest tests/test_replay_gpu.py tests/test_config3_gpu.py tests/test_multirank_gpu.py tests/test_update_gpu.py tests/test_learn32_gpu.py tests/test_actor_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/rf/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/rf/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_learner_prof.sh lp3
