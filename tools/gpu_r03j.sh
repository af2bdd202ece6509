#!/bin/bash
# round 3, pass j: RCCL-in-graph rehearsal test, then the driver's bench command with every leg
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_rccl_capture_gpu.py > gpurun_out/r03j_pytest_rccl.txt 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r03j_pytest_rccl.txt | tail -8
[ $rc -eq 0 ] || { tail -40 gpurun_out/r03j_pytest_rccl.txt; exit 1; }
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03j_bench_k20.json 2> gpurun_out/r03j_bench_k20.err || { echo bench failed; tail -30 gpurun_out/r03j_bench_k20.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r03j_bench_k20.json").read().strip().splitlines()[-1])
print("value %.4g wall_us %.3f ev_us %.3f frac %.3f" % (d["value"], d["ms_per_step"] * 1e3, d["config"]["event_ms_per_step"] * 1e3, d["roofline"]["frac"]), d["episodes"])
for k, v in (d.get("learner") or {}).items():
    if isinstance(v, dict):
        r = v.get("roofline") or {}
        print(k, "ms/tick %.4f" % v["gpu_ms_per_tick"], "dom", r.get("kernel"), "frac %.4f" % r.get("frac", -1), {kk: round(vv["us"], 2) for kk, vv in (r.get("kernels") or {}).items()}, v.get("roofline_error"))
print("errors", d.get("errors"))
PY
