#!/bin/bash
# Round-2 profile refresh: default bench line, its rocprofv3 kernel stats,
# learner piece timings and the actor forward, each step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r02
O=gpurun_out/r02
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
tail -c 600 $O/bench_default.json; echo
timeout -k 10 300 python tools/bench_update_parts.py > $O/update_parts.jsonl 2>/dev/null || exit $?
timeout -k 10 120 python tools/bench_actor_fwd.py > $O/actor_fwd.jsonl 2>/dev/null || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 bench.py --no-learner --no-cpu-baseline > $O/prof_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_update -o run -- python3 tools/bench_update.py --iters 100 > $O/prof_update.log 2>&1 || exit $?
echo done
