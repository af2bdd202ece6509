#!/bin/bash
# round 3, pass h: 512-lane split multi geometry with staggered waves
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_multi_gpu.py > gpurun_out/r03h_pytest.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03h_pytest.txt; exit 1; }
tail -2 gpurun_out/r03h_pytest.txt
timeout -k 10 500 python -u tools/multi_sweep.py --envs 65536 --ticks 20,400 --pols 1 --splits 0 --reps 2 --no-graph > gpurun_out/r03h_sweep.jsonl 2> gpurun_out/r03h_sweep.err || { echo sweep failed; tail gpurun_out/r03h_sweep.err; exit 1; }
timeout -k 10 500 python -u tools/multi_sweep.py --envs 65536,131072 --ticks 20,400 --pols 1 --splits 1 --blocks 512 --staggers 0,1,2,3,4,6 --reps 2 --no-graph >> gpurun_out/r03h_sweep.jsonl 2>> gpurun_out/r03h_sweep.err || { echo sweep failed; tail gpurun_out/r03h_sweep.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r03h_sweep.jsonl'):
    d=json.loads(l); print(d['envs'], 'pol', d['policy'], 'split', d['split'], 'blk', d['block'], 'stag', d['stagger'], 'T', d['ticks_per_launch'], 'us %.3f'%d['us_per_tick'], 'frac %.3f'%d['frac'], 'rep', d['rep'])
"
