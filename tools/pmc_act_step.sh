#!/bin/bash
# MFMA / VALU counters of the config-5 acting launch (k_act_step32<true>,
# 65,536 games, parameter noise) and config 3's (4,096 games, action noise):
# two --pmc passes each (tools/pmc_act_step.py), summarised by
# tools/pmc_summary.py.   bash tools/pmc_act_step.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
TAG=${1:-pa}; OUT=gpurun_out/pmca_$TAG; mkdir -p $OUT
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAVES"
for G in "65536 param" "4096 action"; do
  set -- $G
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    D=$OUT/g$1_$2_p$i
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $D -o pmc \
      -- python3 tools/pmc_act_step.py --games $1 --noise $2 --launches 30 > $D.log 2>&1 || { echo "pmc $G $i failed"; tail -3 $D.log; exit 1; }
  done
done
python3 tools/pmc_summary.py $(find $OUT -name "*counter_collection.csv" | sort) > $OUT/summary.json
python3 - $OUT/summary.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k in d["kernels"]:
    if "act_step" not in k["kernel"]:
        continue
    c = k["counters"]
    print(k["source"].split("/")[-3], k["kernel"], "grid", k["grid"], "us", k["median_us"], "mfma_util", k["mfma_util_chip"],
          {x: c[x] for x in sorted(c)})
PY
