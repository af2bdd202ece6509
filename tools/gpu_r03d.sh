#!/bin/bash
# round 3, pass d: unrolled multi kernels (action prefetch): parity, sweep, short region, bench K=20
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_multi_gpu.py tests/test_bench_path_gpu.py > gpurun_out/r03d_pytest.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03d_pytest.txt; exit 1; }
tail -2 gpurun_out/r03d_pytest.txt
timeout -k 10 300 python -u tools/multi_sweep.py --envs 8192,32768,65536,131072 --ticks 20,400 --pols 1,0 --splits 0,1 --reps 2 --no-graph > gpurun_out/r03d_sweep.jsonl 2> gpurun_out/r03d_sweep.err || { echo sweep failed; tail gpurun_out/r03d_sweep.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r03d_sweep.jsonl'):
    d=json.loads(l); print(d['envs'], 'pol', d['policy'], 'split', d['split'], 'T', d['ticks_per_launch'], 'us %.3f'%d['us_per_tick'], 'frac %.3f'%d['frac'], 'rep', d['rep'])
"
timeout -k 10 120 python -u tools/short_run_multi.py --k 20 --reps 30 > gpurun_out/r03d_short.json 2> gpurun_out/r03d_short.err || { echo short failed; tail gpurun_out/r03d_short.err; exit 1; }
cat gpurun_out/r03d_short.json
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-learner --no-cpu-baseline --no-large --no-full --no-rollout --no-variants > gpurun_out/r03d_bench_k20_$i.json 2> gpurun_out/r03d_bench_k20_$i.err || { echo bench20 failed; tail -20 gpurun_out/r03d_bench_k20_$i.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r03d_bench_k20_$i.json').read().strip().splitlines()[-1]); print('K20 value %.4g wall_us/step %.3f ev_us/step %.3f frac %.3f'%(d['value'], d['ms_per_step']*1e3, d['config']['event_ms_per_step']*1e3, d['roofline']['frac']), d['episodes'])"
done
