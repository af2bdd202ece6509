#!/bin/bash
# One gpurun session: GPU parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; any fault/abort/timeout exit status
# (anything other than 0 or an ordinary pytest failure 1) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r01}
STEPS=${STEPS:-all}

stop_if_fault() {  # $1 = exit code, $2 = step name
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then
    echo "STEP $2 ended with status $1: stopping (no further GPU steps)"; exit "$1"
  fi
}

rocm-smi --showproductname > $OUT/rocm_smi.txt 2>&1 || true
python -c "import skillshot_learning_amd as s; s.load_library(); print('lib ok')" || exit 3

if [[ "$STEPS" == all || "$STEPS" == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
  rc=$?; tail -25 $OUT/pytest_gpu_$TAG.log; stop_if_fault $rc pytest
fi
if [[ "$STEPS" == all || "$STEPS" == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1
  rc=$?; tail -3 $OUT/smoke_$TAG.log; stop_if_fault $rc smoke
fi
if [[ "$STEPS" == all || "$STEPS" == *bench* ]]; then
  timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
  rc=$?; cat $OUT/bench_$TAG.json; tail -5 $OUT/bench_$TAG.err; stop_if_fault $rc bench
fi
if [[ "$STEPS" == all || "$STEPS" == *prof* ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run \
    -- python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline --no-large --no-learner > $OUT/prof_bench_$TAG.json 2> $OUT/prof_$TAG.err
  rc=$?; tail -3 $OUT/prof_$TAG.err; stop_if_fault $rc rocprof
  find $OUT/prof_$TAG -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_$TAG.csv \; 2>/dev/null
  head -20 $OUT/kernel_stats_$TAG.csv 2>/dev/null
fi
echo "gpu_check done"
