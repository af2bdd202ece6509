#!/bin/bash
# HBM traffic per launch (rocprofv3 FETCH_SIZE / WRITE_SIZE passes, each its
# own run, gfx950 corrections in tools/pmc_parse.py) of the headline k_step
# and of the full-contract k_step_split (obs + reward): bash tools/gpu_traffic.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=${1:-tr}; O=gpurun_out
for leg in "k_step:" "k_step_split:--obs"; do
  K=${leg%%:*}; F=${leg#*:}
  for C in FETCH_SIZE WRITE_SIZE; do
    D=$O/pmc_${TAG}_${K}_$C
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $D -o pmc \
      -- python3 tools/pmc_run.py --envs 65536 --launches 300 $F > $D.log 2>&1 || { echo "pmc $K $C failed"; tail -3 $D.log; exit 1; }
  done
  B=193; [ "$K" = k_step_split ] && B=297
  python3 tools/pmc_parse.py --kernel $K --envs 65536 --bytes-per-env $B $O/pmc_${TAG}_${K}_* --write $O/traffic_${K}_$TAG.json
done
