#!/bin/bash
# sliced fp32 gradient kernels: parity against the Keras restatement, then per-piece timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_learn32_gpu.py > gpurun_out/r03v_pytest_learn32.txt 2>&1 || { tail -30 gpurun_out/r03v_pytest_learn32.txt; exit 1; }
tail -3 gpurun_out/r03v_pytest_learn32.txt
timeout -k 10 300 python -u tools/bench_update_parts.py --precisions fp32 --batches 256,512 --slices 1 > gpurun_out/r03v_update_parts.jsonl 2>&1 || { tail -30 gpurun_out/r03v_update_parts.jsonl; exit 1; }
cat gpurun_out/r03v_update_parts.jsonl
timeout -k 10 600 python -u bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-large --no-full --no-rollout --no-variants > gpurun_out/r03v_bench_learner.json 2> gpurun_out/r03v_bench_learner.err || { tail -20 gpurun_out/r03v_bench_learner.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r03v_bench_learner.json").read().strip().splitlines()[-1])
for k, v in d.get("learner", {}).items():
    if isinstance(v, dict):
        print(k, v.get("ms_per_tick"), v.get("gpu_ms_per_tick"), {kk: vv.get("us") for kk, vv in v.get("roofline", {}).get("kernels", {}).items()})
PY
