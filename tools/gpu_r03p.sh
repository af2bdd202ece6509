#!/bin/bash
# kernel-trace stats of the sliced fp32 update pieces at batch 256
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03p_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_update_parts.py --precisions fp32 --batches 256 --slices 1 > $GRAFT_REPO_ROOT/gpurun_out/r03p_log.txt 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r03p_log.txt; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/r03p_prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
