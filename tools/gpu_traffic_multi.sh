#!/bin/bash
# HBM traffic of k_step_multi (FETCH_SIZE / WRITE_SIZE passes, each its own
# run, gfx950 corrections in tools/pmc_parse.py) for both state ports at
# 65,536 games, 20 ticks per launch: bash tools/gpu_traffic_multi.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=${1:-tr}; O=gpurun_out; T=20
for POL in 1 0; do
  for C in FETCH_SIZE WRITE_SIZE; do
    D=$O/pmc_${TAG}_multi${POL}_$C
    SK_MULTI_POLICY=$POL timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $D -o pmc \
      -- python3 tools/pmc_run.py --envs 65536 --launches 60 --ring 400 --multi $T > $D.log 2>&1 || { echo "pmc multi$POL $C failed"; tail -3 $D.log; exit 1; }
  done
  python3 tools/pmc_parse.py --kernel k_step_multi --envs 65536 --bytes-per-env 193 --ticks-per-launch $T \
    $O/pmc_${TAG}_multi${POL}_* --write $O/traffic_k_step_multi_pol${POL}_$TAG.json
done
