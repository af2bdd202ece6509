#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each, within the per-pass block
# limits) over tools/bench_mlp_kernels.py --eager for one MLP kernel:
#   bash tools/pmc_kernel.sh actor_noise 131072 TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
K=${1:-actor_noise}; ROWS=${2:-131072}; TAG=${3:-$K}
OUT=gpurun_out/pmck_$TAG; mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAVES"
P3="SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_MISC"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o pmc -- python3 tools/bench_mlp_kernels.py --eager --only $K --rows $ROWS --reps 20 > /dev/null 2>$OUT/p$i.err || exit $?
done
echo done
