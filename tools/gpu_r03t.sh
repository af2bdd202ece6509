#!/bin/bash
# the whole GPU suite and smoke on the current tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03t; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.txt; tail -2 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
