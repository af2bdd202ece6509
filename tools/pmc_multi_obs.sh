#!/bin/bash
# SQ counter passes over the full-contract multi-tick kernel
# (sk_env_step_multi_obs -> k_step_split_multi<1, *, true>; tools/pmc_run.py
# --multi-obs 20, 65,536 games) beside the headline k_step_multi: where a
# tick's wave-cycles go (parked on memory vs issuing VALU).
#   bash tools/pmc_multi_obs.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
TAG=${1:-pmo}; OUT=gpurun_out/pmco_$TAG; mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_WAVES"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_BRANCH"
for MODE in "--multi-obs 20" "--multi 20"; do
  tag=$(echo $MODE | tr -d ' -')
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    D=$OUT/${tag}_p$i
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $D -o pmc \
      -- python3 tools/pmc_run.py --envs 65536 --launches 40 --ring 400 $MODE > $D.log 2>&1 || { echo "pmc $MODE $i failed"; tail -3 $D.log; exit 1; }
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
