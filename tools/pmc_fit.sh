#!/bin/bash
# Counter passes of the resident models_fit kernels (k_fit_critic<16>,
# k_fit_actor<16>, one XCD; tools/bench_fit.py, one rep of resident
# launches of 2,048 steps, --resident-only):
# two --pmc passes of 8 SQ counters each, then tools/pmc_summary.py.
#   bash tools/pmc_fit.sh TAG   -> gpurun_out/pmc_TAG/summary.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
OUT=gpurun_out/pmc_${1:-fit}; mkdir -p $OUT
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  BENCH_FIT_CFG=16:1 timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $OUT/f$i -o pmc \
    -- python3 tools/bench_fit.py --reps 1 --steps 2048 --resident-only > $OUT/f$i.log 2>&1 || { echo "pmc $i failed"; tail -3 $OUT/f$i.log; exit 1; }
done
python3 tools/pmc_summary.py $(find $OUT -name "*counter_collection.csv" | sort) > $OUT/summary.json
echo done
