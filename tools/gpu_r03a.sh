#!/bin/bash
# round 3, first GPU pass: multi-tick parity + bench-path parity + A/B sweep
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_multi_gpu.py tests/test_bench_path_gpu.py > gpurun_out/r03a_pytest.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03a_pytest.txt; exit 1; }
tail -3 gpurun_out/r03a_pytest.txt
timeout -k 10 300 python -u tools/multi_sweep.py --envs 8192,65536,262144 --ticks 1,5,20,100,400 --pols 0,1 --reps 2 > gpurun_out/r03a_sweep.jsonl 2> gpurun_out/r03a_sweep.err
rc=$?; cat gpurun_out/r03a_sweep.jsonl | cut -c1-220; exit $rc
