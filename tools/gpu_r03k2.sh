#!/bin/bash
# the driver's short region with the events recorded inside the launch call
# (sk_env_step_multi_timed, current bench.py) -- 4 runs -- then bench.py's
# N > 1 path rehearsed with 2 gloo ranks on the one GPU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03k2; mkdir -p $O
: > $O/k20.jsonl
for rep in 1 2 3 4; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-learner --no-cpu-baseline --no-large --no-full --no-rollout --no-variants > $O/b.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  python3 -c "
import json; d = json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print(json.dumps(dict(rep=$rep, value=d['value'], wall_us=d['ms_per_step']*1e3, event_us=d['config']['event_ms_per_step']*1e3, frac=d['roofline']['frac'], episodes=d.get('episodes'))))" >> $O/k20.jsonl
done
cat $O/k20.jsonl
bash tools/gpu_2rank_gloo.sh && cp gpurun_out/bench_2rank_gloo.json $O/
