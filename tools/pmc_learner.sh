#!/bin/bash
# MFMA utilisation of the learner kernels: one rocprofv3 --pmc pass (6 SQ
# counters) over tools/bench_update.py and tools/bench_actor_fwd.py.
#   bash tools/pmc_learner.sh   -> gpurun_out/pmcl/{u,f}/pmc_counter_collection.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
OUT=gpurun_out/pmcl; mkdir -p $OUT
P="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_ANY"
timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/u -o pmc -- python3 tools/bench_update.py --iters 20 > $OUT/u.out 2>$OUT/u.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/f -o pmc -- python3 tools/bench_actor_fwd.py --iters 10 > $OUT/f.out 2>$OUT/f.err || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t -o run -- python3 tools/bench_actor_fwd.py --iters 10 > /dev/null 2>&1 || exit $?
echo done
