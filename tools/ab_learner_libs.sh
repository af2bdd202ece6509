#!/bin/bash
# Alternating A/B (3 passes) of prebuilt ab/*.so on the learner tick
# (bench.learner_rate: config 3 and config 5 on one GPU, bf16 and fp32).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-ab_learner_libs}.jsonl; : > $OUT
for r in 1 2 3; do for f in ab/*.so; do n=$(basename $f .so)
  SK_LIB_PATH=$PWD/$f timeout -k 10 300 python3 -c "
import bench, json
for n, ex in ((4096, 'action_noise'), (65536, 'param_noise')):
    for pr in ('fp32', 'bf16'):
        d = bench.learner_rate(n, 1, 0, 200, batch=256, exploration=ex, precision=pr)
        print(json.dumps(dict(lib='$n', round=$r, envs=n, precision=pr, us_per_tick=d['ms_per_tick'] * 1e3)))
" >> $OUT 2> /tmp/abl.err || { tail -5 /tmp/abl.err; exit 3; }
done; done
python3 - $OUT <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l); d[(j["envs"], j["precision"], j["lib"])].append(round(j["us_per_tick"], 1))
for k, v in sorted(d.items()): print(k, v)
PY
