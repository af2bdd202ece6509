#!/bin/bash
# learner legs after the sliced update kernels
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-large --no-full --no-rollout --no-variants > gpurun_out/r03r_bench_learner.json 2> gpurun_out/r03r_bench_learner.err || { tail -20 gpurun_out/r03r_bench_learner.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r03r_bench_learner.json").read().strip().splitlines()[-1])
for k, v in d.get("learner", {}).items():
    if isinstance(v, dict):
        print(k, v.get("ms_per_tick"), v.get("gpu_ms_per_tick"), {kk: vv.get("us") for kk, vv in v.get("roofline", {}).get("kernels", {}).items()})
PY
