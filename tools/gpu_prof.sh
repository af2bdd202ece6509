#!/bin/bash
# Decompose k_step cost: diag floors sweep + rocprofv3 PMC passes (each its own run).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=${1:-prof}
O=gpurun_out
timeout -k 10 300 python tools/sweep.py --variants empty,copy,0,1 --envs 65536,262144 > $O/sweep_diag_$TAG.jsonl 2>$O/sweep_diag_$TAG.err; rc=$?
cat $O/sweep_diag_$TAG.jsonl; [ $rc -ne 0 ] && { tail -5 $O/sweep_diag_$TAG.err; exit $rc; }
rocprofv3 -L > $O/rocprof_counters_list.txt 2>&1 || true
for C in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES" "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  D=$O/pmc_${TAG}_$(echo $C | tr ' ' '_')
  timeout -k 10 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $D -o pmc \
    -- python3 tools/pmc_run.py --envs 65536 --launches 300 > $D.log 2>&1; rc=$?
  echo "pmc [$C] rc=$rc"; tail -2 $D.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
python tools/pmc_parse.py --kernel k_step --envs 65536 $O/pmc_${TAG}_* --write $O/traffic_k_step_$TAG.json
