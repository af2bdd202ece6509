#!/bin/bash
# packed resident form vs the 88-B form across sizes (lane-per-game kernel,
# write-through port, 256-lane workgroups), 20 and 400 ticks per launch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03pk2; mkdir -p $O
: > $O/sweep.jsonl
for pk in 1 0; do
  SK_MULTI_PACK=$pk timeout -k 10 300 python -u tools/multi_sweep.py --envs 32768,65536,131072,262144 --ticks 20,400 --pols 1 --reps 2 --splits 0 2> $O/err.txt | sed "s/^{/{\"pack\": $pk, /" >> $O/sweep.jsonl || { tail -20 $O/err.txt; exit 1; }
done
cat $O/sweep.jsonl
