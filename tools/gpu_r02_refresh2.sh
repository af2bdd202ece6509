#!/bin/bash
# Round-2 refresh after the counter / trig / warm-exec changes: GPU tests,
# smoke, the driver-style short bench, the default bench line and the
# rocprofv3 kernel stats of the headline leg; each step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && T=${1:-r02b}; mkdir -p gpurun_out/$T
O=gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit $?
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 bench.py --no-learner --no-cpu-baseline --no-large --no-full --no-rollout > $O/prof_bench.log 2>&1 || exit $?
T=$T python - <<'PY'
import json, os; T = os.environ["T"]
for f in ("bench_driver", "bench_default"):
    d = json.load(open(f"gpurun_out/{T}/{f}.json"))
    print(f, round(d["value"] / 1e9, 3), "G", "ms/step", d["ms_per_step"], "event", d["config"]["event_ms_per_step"], "frac", round(d["roofline"]["frac"], 3))
PY
echo done
