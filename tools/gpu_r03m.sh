#!/bin/bash
# round 3, pass m: split multi kernel without the packed path (small grids), parity + sweep
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_multi_gpu.py tests/test_bench_path_gpu.py > gpurun_out/r03m_pytest.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03m_pytest.txt; exit 1; }
tail -2 gpurun_out/r03m_pytest.txt
timeout -k 10 500 python -u tools/multi_sweep.py --envs 8192,16384,32768,65536 --ticks 20,400 --pols 1 --splits -1 --reps 2 --no-graph > gpurun_out/r03m_sweep.jsonl 2> gpurun_out/r03m_sweep.err || { echo sweep failed; tail gpurun_out/r03m_sweep.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r03m_sweep.jsonl'):
    d=json.loads(l); print(d['envs'], 'split', d['split'], 'T', d['ticks_per_launch'], 'us %.3f'%d['us_per_tick'], 'frac %.3f'%d['frac'], 'rep', d['rep'])
"
