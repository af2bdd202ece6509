#!/bin/bash
# round 3, pass l: refresh the headline records: PMC traffic of the final
# k_step_multi (both ports), rocprofv3 kernel stats of the headline leg at
# K = 4000 and K = 20, the default bench line with every leg
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/gpu_traffic_multi.sh r03l > gpurun_out/r03l_traffic.log 2>&1 || { echo traffic failed; tail gpurun_out/r03l_traffic.log; exit 1; }
grep -h "traffic_over\|hbm_bytes_per_tick" gpurun_out/traffic_k_step_multi_pol*_r03l.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03l -o prof -- python3 bench.py --no-learner --no-cpu-baseline --no-large --no-full --no-rollout --no-variants > gpurun_out/r03l_prof_bench.json 2> gpurun_out/r03l_prof_bench.err || { echo prof failed; tail -5 gpurun_out/r03l_prof_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03l_k20 -o prof -- python3 bench.py --steps 20 --warmup 5 --no-learner --no-cpu-baseline --no-large --no-full --no-rollout --no-variants > gpurun_out/r03l_prof_bench_k20.json 2> gpurun_out/r03l_prof_bench_k20.err || { echo prof20 failed; tail -5 gpurun_out/r03l_prof_bench_k20.err; exit 1; }
grep -h "multi" gpurun_out/prof_r03l/prof_kernel_stats.csv gpurun_out/prof_r03l_k20/prof_kernel_stats.csv | cut -c1-160
timeout -k 10 900 python3 -u bench.py > gpurun_out/r03l_bench_default.json 2> gpurun_out/r03l_bench_default.err || { echo bench failed; tail -20 gpurun_out/r03l_bench_default.err; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r03l_prof_bench.json", "gpurun_out/r03l_prof_bench_k20.json", "gpurun_out/r03l_bench_default.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, "value %.4g wall_us %.3f ev_us %.3f frac %.3f traffic %s" % (d["value"], d["ms_per_step"] * 1e3, d["config"]["event_ms_per_step"] * 1e3, d["roofline"]["frac"], d["roofline"]["traffic"]), d["episodes"])
d = json.loads(open("gpurun_out/r03l_bench_default.json").read().strip().splitlines()[-1])
for k in ("step_variants", "full_contract_tick", "rollout_random", "large_batch"):
    v = d.get(k)
    print(k, {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in (v or {}).items() if not isinstance(vv, (dict, str))} if isinstance(v, dict) else v)
for k, v in (d.get("learner") or {}).items():
    if isinstance(v, dict):
        r = v.get("roofline") or {}
        print(k, "ms/tick %.4f" % v["gpu_ms_per_tick"], "dom", r.get("kernel"), "frac %.4f" % r.get("frac", -1), "tick_frac %.4f" % r.get("tick_frac", -1))
print("cpu", d.get("cpu_baseline", {}).get("value"), "errors", d.get("errors"))
PY
