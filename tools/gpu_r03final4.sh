#!/bin/bash
# round 3 final records (second pass, after the overlapped ticks and the
# 88-B multi-tick default): PMC traffic of the headline kernel refreshed first
# (the bench line reads it), then the full GPU suite and smoke, rocprofv3 kernel stats
# of the headline leg (K = 4,000 and the driver's K = 20) and of the learner
# ticks (config 3 fp32 / bf16), the default bench line with every leg, the
# driver's command, PMC MFMA utilisation of the learner kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03i; mkdir -p $O
stop() { echo "STEP $1 ended with status $2: stopping"; exit $2; }
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.txt; tail -2 $O/pytest_gpu.txt; [ $rc -le 1 ] || stop pytest $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || stop smoke $?
tail -1 $O/smoke.txt
bash tools/gpu_traffic_multi.sh r03i > $O/traffic.log 2>&1 || stop traffic $?
cp gpurun_out/traffic_k_step_multi_pol1_r03i.json profiles/traffic_k_step_multi.json
cp gpurun_out/traffic_k_step_multi_pol0_r03i.json profiles/traffic_k_step_multi_pol0.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- python3 bench.py --no-learner --no-cpu-baseline --no-large --no-full --no-rollout --no-variants > $O/prof_bench.json 2> $O/prof_bench.err || stop prof $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_k20 -o prof -- python3 bench.py --steps 20 --warmup 5 --no-learner --no-cpu-baseline --no-large --no-full --no-rollout --no-variants > $O/prof_bench_k20.json 2> $O/prof_bench_k20.err || stop prof20 $?
for cfg in "4096 action_noise fp32 c3" "4096 action_noise bf16 c3" "65536 param_noise fp32 c5" "65536 param_noise bf16 c5"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_learn_$4_$3 -o prof -- python3 -c "
import bench, json
r = bench.learner_rate($1, 1, 0, 200, batch=256, exploration='$2', precision='$3')
print(json.dumps(r))" > $O/prof_learn_$4_$3.json 2> $O/prof_learn_$4_$3.err || stop proflearn $?
done
timeout -k 10 900 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || stop bench $?
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_driver_k20.json 2> $O/bench_driver_k20.err || stop bench20 $?
bash tools/pmc_learner.sh > $O/pmc.log 2>&1 || stop pmc $?
python3 tools/pmc_summary.py gpurun_out/pmcl/u/pmc_counter_collection.csv gpurun_out/pmcl/f/pmc_counter_collection.csv > $O/pmc_mfma_learner.json 2> $O/pmc_summary.err || echo "pmc summary failed"
python3 - <<'PY'
import json
for f in ("prof_bench", "prof_bench_k20", "bench_default", "bench_driver_k20"):
    d = json.loads(open(f"gpurun_out/r03i/{f}.json").read().strip().splitlines()[-1])
    print(f, "value %.4g wall_us %.3f ev_us %.3f frac %.3f" % (d["value"], d["ms_per_step"] * 1e3, d["config"]["event_ms_per_step"] * 1e3, d["roofline"]["frac"]), d["episodes"])
d = json.loads(open("gpurun_out/r03i/bench_default.json").read().strip().splitlines()[-1])
for k, v in (d.get("learner") or {}).items():
    if isinstance(v, dict):
        r = v.get("roofline") or {}
        print(k, "ms/tick %.4f" % v["gpu_ms_per_tick"], "dom", r.get("kernel"), "frac %.4f" % r.get("frac", -1))
print("full", (d.get("full_contract_tick") or {}).get("us_per_launch"), "cpu", (d.get("cpu_baseline") or {}).get("value"), "errors", d.get("errors"))
PY
