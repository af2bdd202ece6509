#!/bin/bash
# LDS layouts of the sliced update kernels (k_grad_slice_fwd / _bwd), new
# (default build) against the padded row-major ones (a -DSK_SL_SWZ=0 variant;
# OLD= names another variant, e.g. -DSK_BWD_HALVES=1):
#  * bit identity of the nets, targets and ring after a graph-replayed learner
#    run (tools/learner_bits.py), the layouts must not change the arithmetic;
#  * LDS instruction and bank-conflict counters and the MFMA / wait counters
#    (two --pmc passes over tools/bench_update.py at batch 256);
#  * per-piece device time (tools/bench_update_parts.py).
#   tools/build_variant.sh gpuab/swz0.so -DSK_SL_SWZ=0
#   bash tools/lds_ab.sh TAG     -> gpurun_out/lds_TAG/...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/lds_${1:-ab}; mkdir -p $OUT
OLD=${OLD:-$PWD/gpuab/swz0.so}  # any variant build: OLD=$PWD/gpuab/h1.so for the one-workgroup backward
[ -f "$OLD" ] || { echo "missing $OLD"; exit 1; }
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAVES"
for V in new old; do
  if [ $V = old ]; then export SK_LIB_PATH=$OLD; else unset SK_LIB_PATH; fi
  timeout -k 10 180 python3 tools/learner_bits.py --out $OUT/bits_$V.npz > $OUT/bits_$V.log 2>&1 \
    || { echo "bits $V failed"; tail -3 $OUT/bits_$V.log; exit 1; }
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $OUT/${V}_u$i -o pmc \
      -- python3 tools/bench_update.py --batches 256 --iters 20 > $OUT/${V}_u$i.log 2>&1 \
      || { echo "pmc $V $i failed"; tail -3 $OUT/${V}_u$i.log; exit 1; }
  done
done
for r in 1 2; do
  for V in new old; do
    if [ $V = old ]; then export SK_LIB_PATH=$OLD; else unset SK_LIB_PATH; fi
    timeout -k 10 180 python3 tools/bench_update_parts.py --batches 256 --precisions fp32 \
      | sed "s/^{/{\"lib\": \"$V\", \"rep\": $r, /" >> $OUT/parts.jsonl || { echo "parts $V failed"; exit 1; }
  done
done
unset SK_LIB_PATH
python3 tools/learner_bits.py --compare $OUT/bits_new.npz $OUT/bits_old.npz > $OUT/bits_compare.txt 2>&1
echo "bits compare rc $?"; cat $OUT/bits_compare.txt
for V in new old; do
  python3 tools/pmc_summary.py $(find $OUT/${V}_u1 $OUT/${V}_u2 -name "*counter_collection.csv" | sort) > $OUT/summary_$V.json
done
echo done
