# Config-5 acting launch (k_act_step32<true>, 65,536 games, parameter noise)
# per library variant under rocprofv3 --kernel-trace --stats: 3 vs 4
# workgroups per CU (profiles/r05zn_act_occupancy_ab.jsonl).  Variants, built
# beforehand with the SK_ACT_LDX1 macro of that experiment (not kept):
#   tools/build_variant.sh ab_run/base.so
#   tools/build_variant.sh ab_run/w4.so -DSK_ACT_WAVES=4 -DSK_ACT_LDX1=16
#   tools/build_variant.sh ab_run/x16.so -DSK_ACT_LDX1=16
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for v in base w4 x16 base w4; do
  SK_LIB_PATH=$PWD/ab_run/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/actab/$v -o run --output-format csv -- python3 tools/pmc_act_step.py --games 65536 --launches 30 > gpurun_out/actab_$v.log 2>&1
  f=$(find gpurun_out/actab/$v -name "*kernel_stats.csv" | head -1)
  grep -h "k_act_step32" "$f" | sed "s/^/$v,/" >> gpurun_out/actab_summary.csv
  rm -rf gpurun_out/actab/$v
done
