#!/bin/bash
# sliced fp32 gradient kernels: parity against the Keras restatement, then per-piece timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_learn32_gpu.py > gpurun_out/r03q_pytest_learn32.txt 2>&1 || { tail -30 gpurun_out/r03q_pytest_learn32.txt; exit 1; }
tail -3 gpurun_out/r03q_pytest_learn32.txt
timeout -k 10 300 python -u tools/bench_update_parts.py --precisions fp32 --batches 256,512 --slices 1 > gpurun_out/r03q_update_parts.jsonl 2>&1 || { tail -30 gpurun_out/r03q_update_parts.jsonl; exit 1; }
cat gpurun_out/r03q_update_parts.jsonl
