#!/bin/bash
# Quick GPU pass after a step-kernel change: the step parity tests, then the
# bench line without the CPU baseline / large-batch legs; each step under its
# own limit, chained so a fault ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
T=${1:-quick}; O=gpurun_out/$T; mkdir -p $O
TESTS=${TESTS:-tests/test_gpu_parity.py}
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python bench.py --no-cpu-baseline --no-large ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
T=$T python - <<'PY'
import json, os
d = json.load(open(f"gpurun_out/{os.environ['T']}/bench.json"))
print("headline", round(d["value"] / 1e9, 3), "G event us", round(d["config"]["event_ms_per_step"] * 1e3, 3), "frac", round(d["roofline"]["frac"], 3))
f = d.get("full_contract_tick") or {}
print("full", f.get("us_per_launch"), (f.get("roofline") or {}).get("frac"))
for k, v in (d.get("learner") or {}).items():
    if isinstance(v, dict) and "ms_per_tick" in v:
        print(k, round(v["ms_per_tick"] * 1e3, 2), "us/tick", round(v["env_steps_per_s"] / 1e6, 1), "M/s")
PY
