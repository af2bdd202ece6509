#!/bin/bash
# round 3, pass k: DPP pair swaps in the split kernels; kernel-attached bench events
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_multi_gpu.py tests/test_bench_path_gpu.py > gpurun_out/r03k_pytest.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03k_pytest.txt; exit 1; }
tail -2 gpurun_out/r03k_pytest.txt
timeout -k 10 500 python -u tools/multi_sweep.py --envs 8192,32768,65536 --ticks 20,400 --pols 1 --splits 0,1 --reps 2 --no-graph > gpurun_out/r03k_sweep.jsonl 2> gpurun_out/r03k_sweep.err || { echo sweep failed; tail gpurun_out/r03k_sweep.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r03k_sweep.jsonl'):
    d=json.loads(l); print(d['envs'], 'split', d['split'], 'T', d['ticks_per_launch'], 'us %.3f'%d['us_per_tick'], 'frac %.3f'%d['frac'], 'rep', d['rep'])
"
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-learner --no-cpu-baseline --no-large --no-full --no-rollout > gpurun_out/r03k_bench_k20_$i.json 2> gpurun_out/r03k_bench_k20_$i.err || { echo bench20 failed; tail -20 gpurun_out/r03k_bench_k20_$i.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r03k_bench_k20_$i.json').read().strip().splitlines()[-1]); print('K20 value %.4g wall_us/step %.3f ev_us/step %.3f frac %.3f'%(d['value'], d['ms_per_step']*1e3, d['config']['event_ms_per_step']*1e3, d['roofline']['frac']), d['episodes'], {k:(round(v['us_per_tick'],3) if isinstance(v,dict) else None) for k,v in d['step_variants'].items()})"
done
