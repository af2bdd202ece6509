#!/bin/bash
# the whole GPU suite and smoke on the current tree, then the Adam sizing A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
bash tools/gpu_r03t.sh && cp gpurun_out/r03t/pytest_gpu.txt gpurun_out/r03t/pytest_gpu_v2.txt && bash tools/gpu_r03adp.sh
