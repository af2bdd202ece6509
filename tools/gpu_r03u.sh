#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_actor_fwd.py --precisions fp32 --fwd16 0,1 --rows 256,2048,8192,32768 > gpurun_out/r03u_actor_fwd.jsonl 2>&1 || { tail -20 gpurun_out/r03u_actor_fwd.jsonl; exit 1; }
cat gpurun_out/r03u_actor_fwd.jsonl
