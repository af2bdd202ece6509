#!/bin/bash
# round 3, pass i: multi kernel tick variants (fp32 fast tick, early restart draw)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_multi_gpu.py > gpurun_out/r03i_pytest.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03i_pytest.txt; exit 1; }
tail -2 gpurun_out/r03i_pytest.txt
timeout -k 10 500 python -u tools/multi_sweep.py --envs 65536,131072,262144 --ticks 20,400 --pols 1 --splits 0 --fasts 0,1 --earlys 0,1 --reps 2 --no-graph > gpurun_out/r03i_sweep.jsonl 2> gpurun_out/r03i_sweep.err || { echo sweep failed; tail gpurun_out/r03i_sweep.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r03i_sweep.jsonl'):
    d=json.loads(l); print(d['envs'], 'pol', d['policy'], 'fast', d['fast'], 'early', d['early'], 'T', d['ticks_per_launch'], 'us %.3f'%d['us_per_tick'], 'frac %.3f'%d['frac'], 'rep', d['rep'])
"
