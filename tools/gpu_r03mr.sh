#!/bin/bash
# the fused overlapped tick with multi_rank "grad": the multi-rank GPU tests
# (2 gloo ranks on one GPU; world-size-1 RCCL full / segmented / plain) and
# bench's N > 1 path rehearsed with 2 gloo ranks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03mr; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py tests/test_rccl_capture_gpu.py tests/test_replay_gpu.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; grep -E "^(FAILED|ERROR)" $O/pytest.txt; tail -2 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_2rank_gloo.sh && cp gpurun_out/bench_2rank_gloo.json $O/
