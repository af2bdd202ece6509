#!/bin/bash
# One parametrised GPU session (replaces the round-3 one-off gpu_r03*.sh).
#
#   tools/gpu_run.sh TAG            # on the box, via gpurun
#   STEPS=tests,smoke,bench20 tools/gpu_run.sh r04a
#
# STEPS (comma-separated, run in this order, each under its own timeout,
# the session stops at the first failing step):
#   tests      pytest -m gpu (TESTS= to narrow, e.g. TESTS="tests/test_multi_gpu.py")
#   smoke      __graft_entry__.smoke()
#   traffic    PMC FETCH/WRITE passes of the headline kernel -> profiles/traffic_k_step_multi*.json
#   trafficobs the same for the full-contract multi-tick kernel -> traffic_k_step_split_multi_obs.json
#   prof       rocprofv3 --kernel-trace --stats of the headline leg, K = 4,000 and the driver's K = 20
#   proffull   rocprofv3 --kernel-trace --stats of the headline and full-contract legs (K = 4,000)
#   proflearn  rocprofv3 kernel stats of the learner ticks (config 3 / 5, fp32 / bf16)
#   bench      python bench.py (every leg)                        -> $O/bench_default.json
#   bench20    python bench.py --steps 20 --warmup 5 (the driver)  -> $O/bench_driver_k20.json
#   pmclearn   PMC MFMA utilisation of the learner kernels
#   pmcact     PMC MFMA / VALU / wait counters of the acting launch (tools/pmc_act_step.sh)
#   pmcobs     SQ counters of the full-contract and headline multi-tick kernels (tools/pmc_multi_obs.sh)
#   py:FILE    python3 FILE (a diagnostic script; ARGS= passed through)
# Outputs under gpurun_out/$TAG; copy what is judged into profiles/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:?tag}
O=gpurun_out/$TAG; mkdir -p $O
STEPS=${STEPS:-tests,smoke,bench20}
stop() { echo "STEP $1 ended with status $2: stopping"; exit $2; }
summ() {
python3 - "$O" "$@" <<'PY'
import json, sys
o = sys.argv[1]
for f in sys.argv[2:]:
    try:
        d = json.loads(open(f"{o}/{f}.json").read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable:", e); continue
    print(f, "value %.4g wall_us %.3f ev_us %.3f frac %.3f" % (d["value"], d["ms_per_step"] * 1e3,
          d["config"]["event_ms_per_step"] * 1e3, d["roofline"]["frac"]), d.get("episodes"))
    for k, v in (d.get("learner") or {}).items():
        if isinstance(v, dict):
            r = v.get("roofline") or {}
            print(" ", k, "ms/tick %.4f" % v.get("gpu_ms_per_tick", -1), v.get("tick_mode"), "dom", r.get("kernel"),
                  "frac %.4f" % r.get("frac", -1))
    fc = d.get("full_contract_tick") or {}
    print("  full", fc.get("us_per_launch"), (fc.get("roofline") or {}).get("frac"), "cpu",
          (d.get("cpu_baseline") or {}).get("value"), "errors", d.get("errors"))
PY
}
IFS=, read -ra S <<< "$STEPS"
for s in "${S[@]}"; do
  echo "== $s $(date +%T)"
  case $s in
  tests)
    timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -q -p no:cacheprovider --timeout 240 \
      --timeout-method thread > $O/pytest_gpu.txt 2>&1
    rc=$?; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.txt; tail -2 $O/pytest_gpu.txt; [ $rc -le 1 ] || stop tests $rc
    [ $rc -eq 0 ] || echo "TESTS FAILED (rc $rc)";;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || stop smoke $?
    tail -1 $O/smoke.txt;;
  traffic)
    bash tools/gpu_traffic_multi.sh $TAG > $O/traffic.log 2>&1 || stop traffic $?
    cp gpurun_out/traffic_k_step_multi_pol1_$TAG.json $O/traffic_k_step_multi.json
    cp gpurun_out/traffic_k_step_multi_pol0_$TAG.json $O/traffic_k_step_multi_pol0.json;;
  trafficobs)
    bash tools/gpu_traffic_multi_obs.sh $TAG > $O/traffic_obs.log 2>&1 || stop trafficobs $?
    cp gpurun_out/traffic_k_step_split_multi_obs_$TAG.json $O/traffic_k_step_split_multi_obs.json;;
  prof)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- python3 bench.py \
      --no-learner --no-cpu-baseline --no-large --no-full --no-rollout --no-variants > $O/prof_bench.json \
      2> $O/prof_bench.err || stop prof $?
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_k20 -o prof -- python3 bench.py \
      --steps 20 --warmup 5 --no-learner --no-cpu-baseline --no-large --no-full --no-rollout --no-variants \
      > $O/prof_bench_k20.json 2> $O/prof_bench_k20.err || stop prof20 $?
    summ prof_bench prof_bench_k20;;
  proffull)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_full -o prof -- python3 bench.py \
      --no-learner --no-cpu-baseline --no-large --no-rollout --no-variants > $O/prof_full_bench.json \
      2> $O/prof_full_bench.err || stop proffull $?
    summ prof_full_bench;;
  proflearn)
    for cfg in ${LEARN_CFGS:-"4096:action_noise:fp32:c3" "4096:action_noise:bf16:c3" "65536:param_noise:fp32:c5" "65536:param_noise:bf16:c5"}; do
      IFS=: read -r n ex pr tg <<< "$cfg"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_learn_${tg}_$pr -o prof -- \
        python3 -c "
import bench, json
r = bench.learner_rate($n, 1, 0, 200, batch=256, exploration='$ex', precision='$pr')
print(json.dumps(r))" > $O/prof_learn_${tg}_$pr.json 2> $O/prof_learn_${tg}_$pr.err || stop proflearn $?
    done;;
  bench)
    timeout -k 10 900 python3 -u bench.py ${BENCH_ARGS:-} > $O/bench_default.json 2> $O/bench_default.err || stop bench $?
    summ bench_default;;
  bench20)
    timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $O/bench_driver_k20.json \
      2> $O/bench_driver_k20.err || stop bench20 $?
    summ bench_driver_k20;;
  pmclearn)
    bash tools/pmc_learner.sh > $O/pmc.log 2>&1 || stop pmc $?
    python3 tools/pmc_summary.py gpurun_out/pmcl/u/pmc_counter_collection.csv gpurun_out/pmcl/f/pmc_counter_collection.csv \
      > $O/pmc_mfma_learner.json 2> $O/pmc_summary.err || echo "pmc summary failed";;
  pmcact)
    bash tools/pmc_act_step.sh $TAG > $O/pmc_act.log 2>&1 || stop pmcact $?
    cp gpurun_out/pmca_$TAG/summary.json $O/pmc_act_step.json;;
  pmcobs)
    bash tools/pmc_multi_obs.sh $TAG > $O/pmc_obs.log 2>&1 || stop pmcobs $?
    cp gpurun_out/pmco_$TAG/summary.json $O/pmc_sq_multi_obs.json;;
  py:*)
    f=${s#py:}; b=$(basename $f .py)
    timeout -k 10 ${PYTIMEOUT:-600} python3 -u $f ${ARGS:-} > $O/$b.out 2> $O/$b.err || stop $s $?
    tail -${TAILN:-20} $O/$b.out;;
  *) echo "unknown step $s"; exit 2;;
  esac
done
echo "== done $(date +%T)"
