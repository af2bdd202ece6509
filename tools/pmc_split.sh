#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each) over eager step launches
# with obs (tools/pmc_run.py --obs) for every prebuilt ab/*.so, then the
# per-dispatch summary of k_step_split:  bash tools/pmc_split.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES"
for f in ab/*.so; do n=$(basename $f .so); OUT=gpurun_out/pmcs_$n; mkdir -p $OUT; i=0
  for P in "$P1" "$P2"; do i=$((i+1))
    SK_STEP_VARIANT=${VARIANT:-1} SK_LIB_PATH=$PWD/$f timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o pmc \
      -- python3 tools/pmc_run.py --obs --launches 200 > /dev/null 2>$OUT/p$i.err || exit $?
  done
  echo "== $n"; python3 tools/pmc_sum.py $OUT ${KERNEL:-k_step_split}
done
