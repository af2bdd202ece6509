#!/bin/bash
# 2-rank rehearsal of bench.py's N > 1 path on one GPU (gloo backend, both
# ranks on device 0): strong headline, weak leg, config-4/5 learner legs in
# child process groups.  The hardware RCCL run is the driver's.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
SK_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 2 --steps 200 --warmup 20 --no-large \
  --learner-ticks 40 > gpurun_out/bench_2rank_gloo.json 2> gpurun_out/bench_2rank_gloo.err || { tail -20 gpurun_out/bench_2rank_gloo.err; exit 1; }
python3 -c "
import json; d = json.loads(open('gpurun_out/bench_2rank_gloo.json').read().strip().splitlines()[-1])
print(d['value'] / 1e9, d['n_gpus'], d.get('errors'))
for k, v in (d.get('learner') or {}).items():
    if isinstance(v, dict): print(k, v.get('ms_per_tick'), v.get('capture_attempts'), v.get('multi_rank'), v.get('tick_mode'))
"
