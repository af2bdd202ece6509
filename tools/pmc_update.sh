export TMPDIR=/tmp; mkdir -p gpurun_out/pmcu
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAVES"
P3="SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_SMEM"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmcu/p$i -o pmc -- python3 tools/bench_mlp_kernels.py --eager --only critic_grad_boot --rows 4096 --reps 30 > /dev/null 2>gpurun_out/pmcu/p$i.err || exit $?
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmcu/a$i -o pmc -- python3 tools/bench_mlp_kernels.py --eager --only actor_grad --rows 4096 --reps 30 > /dev/null 2>gpurun_out/pmcu/a$i.err || exit $?
done
find gpurun_out/pmcu -name "*counter_collection.csv" | head
