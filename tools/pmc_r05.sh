#!/bin/bash
# Round-5 counter and trace passes:
#  * MFMA / VALU counters of the learner update chain (k_grad_slice_*,
#    k_adam_flat; tools/bench_update.py at batch 256, both precisions), two
#    --pmc passes;
#  * kernel-trace stats of the config-5 acting launch at 65,536 games with
#    parameter noise (k_act_step32<true>) and with action noise
#    (k_act_step32<false>): the noise's share of the launch.
#   bash tools/pmc_r05.sh TAG   -> gpurun_out/pmc_TAG/...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
OUT=gpurun_out/pmc_${1:-r05}; mkdir -p $OUT
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $OUT/u$i -o pmc \
    -- python3 tools/bench_update.py --batches 256 --iters 20 > $OUT/u$i.log 2>&1 || { echo "pmc $i failed"; tail -3 $OUT/u$i.log; exit 1; }
done
for N in param action; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t_$N -o run \
    -- python3 tools/pmc_act_step.py --games 65536 --noise $N --launches 30 > $OUT/t_$N.log 2>&1 || { echo "trace $N failed"; tail -3 $OUT/t_$N.log; exit 1; }
done
python3 tools/pmc_summary.py $(find $OUT -name "*counter_collection.csv" | sort) > $OUT/summary.json
echo done
