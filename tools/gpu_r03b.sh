#!/bin/bash
# round 3, pass b: bench (default and the driver's K=20), PMC traffic of
# k_step_multi, rocprofv3 kernel-trace stats of the headline leg
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03b_bench_k20.json 2> gpurun_out/r03b_bench_k20.err || { echo bench20 failed; tail -20 gpurun_out/r03b_bench_k20.err; exit 1; }
cut -c1-900 gpurun_out/r03b_bench_k20.json
timeout -k 10 300 python -u bench.py --no-learner --no-cpu-baseline --no-large --no-full --no-rollout > gpurun_out/r03b_bench_default.json 2> gpurun_out/r03b_bench_default.err || { echo bench failed; tail -20 gpurun_out/r03b_bench_default.err; exit 1; }
cut -c1-900 gpurun_out/r03b_bench_default.json
bash tools/gpu_traffic_multi.sh r03b || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03b -o prof -- python3 bench.py --no-learner --no-cpu-baseline --no-large --no-full --no-rollout --no-variants > gpurun_out/r03b_prof_bench.json 2> gpurun_out/r03b_prof_bench.err || { echo prof failed; tail -5 gpurun_out/r03b_prof_bench.err; exit 1; }
find gpurun_out/prof_r03b -name "*kernel_stats.csv" | head -2
