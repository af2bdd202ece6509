#!/bin/bash
# HBM traffic of the full-contract multi-tick kernel (sk_env_step_multi_obs,
# k_step_split_multi<1, *, true>) at 65,536 games, 20 ticks per launch, a
# 64-slab output ring: FETCH_SIZE / WRITE_SIZE passes (each its own run,
# gfx950 corrections in tools/pmc_parse.py):  bash tools/gpu_traffic_multi_obs.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=${1:-tr}; O=gpurun_out; T=20
for C in FETCH_SIZE WRITE_SIZE; do
  D=$O/pmc_${TAG}_multiobs_$C
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $D -o pmc \
    -- python3 tools/pmc_run.py --envs 65536 --launches 60 --ring 400 --multi-obs $T > $D.log 2>&1 || { echo "pmc multiobs $C failed"; tail -3 $D.log; exit 1; }
done
python3 tools/pmc_parse.py --kernel k_step_split_multi --envs 65536 --bytes-per-env 297 --ticks-per-launch $T \
  $O/pmc_${TAG}_multiobs_* --write $O/traffic_k_step_split_multi_obs_$TAG.json
