#!/bin/bash
# SQ counter passes over k_step_multi (tools/pmc_run.py --multi 20, 65,536
# games) for the geometry / port / resident-form variants: where a tick's
# wave-cycles go (waiting on memory vs issuing VALU).  bash tools/pmc_multi.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
TAG=${1:-pm}; OUT=gpurun_out/pmcm_$TAG; mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_WAVES"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_BRANCH"
# VARIANTS: "POL SPLIT PACK" triples (default: round 3's four)
IFS=, read -ra VS <<< "${VARIANTS:-1 0 1,1 1 1,1 0 0,0 0 1}"
for V in "${VS[@]}"; do
  set -- $V; POL=$1; SPL=$2; PK=$3
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    D=$OUT/pol${POL}_split${SPL}_pack${PK}_p$i
    SK_MULTI_POLICY=$POL SK_MULTI_SPLIT=$SPL SK_MULTI_PACK=$PK timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $D -o pmc \
      -- python3 tools/pmc_run.py --envs 65536 --launches 40 --ring 400 --multi 20 > $D.log 2>&1 || { echo "pmc $V $i failed"; tail -3 $D.log; exit 1; }
  done
done
python3 tools/pmc_summary.py $(find $OUT -name "*counter_collection.csv" | sort) > $OUT/summary.json
python3 - $OUT/summary.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k in d["kernels"]:
    if "multi" not in k["kernel"]:
        continue
    c = k["counters"]
    print(k["source"].split("/")[-3], k["kernel"], "us", k["median_us"], {x: c[x] for x in sorted(c)})
PY
