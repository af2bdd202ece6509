#!/bin/bash
# round 3, pass f: packed resident planes in the multi-tick kernels: parity + A/B
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_multi_gpu.py tests/test_bench_path_gpu.py > gpurun_out/r03f_pytest.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03f_pytest.txt; exit 1; }
tail -2 gpurun_out/r03f_pytest.txt
for PK in 1 0; do
SK_MULTI_PACK=$PK timeout -k 10 400 python -u tools/multi_sweep.py --envs 8192,32768,65536,131072 --ticks 20,400 --pols 1,0 --splits -1 --reps 2 --no-graph > gpurun_out/r03f_sweep_pack$PK.jsonl 2> gpurun_out/r03f_sweep.err || { echo sweep failed; tail gpurun_out/r03f_sweep.err; exit 1; }
done
python3 -c "
import json
for pk in (1,0):
  for l in open('gpurun_out/r03f_sweep_pack%d.jsonl'%pk):
    d=json.loads(l); print('pack', pk, d['envs'], 'pol', d['policy'], 'T', d['ticks_per_launch'], 'us %.3f'%d['us_per_tick'], 'frac %.3f'%d['frac'], 'rep', d['rep'])
"
