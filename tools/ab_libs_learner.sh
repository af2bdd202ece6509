#!/bin/bash
# Alternating A/B of prebuilt library variants (ab_run/*.so, SK_LIB_PATH) on
# the learner's reference-order tick (bench.learner_rate) and its launch sets
# (the roofline's acting / critic_step / actor_step times):
#   PASSES=3 CFGS="4096:action_noise" bash tools/ab_libs_learner.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
OUT=gpurun_out/${1:-ab_libs_learner}.jsonl; : > $OUT
for r in $(seq ${PASSES:-3}); do for f in ab_run/*.so; do n=$(basename $f .so)
  SK_LIB_PATH=$PWD/$f timeout -k 10 300 python3 -c "
import bench, json
for cfg in '${CFGS:-4096:action_noise}'.split():
    envs, ex = cfg.split(':')
    d = bench.learner_rate(int(envs), 1, 0, 200, batch=256, exploration=ex, precision='fp32')
    k = {key: round(v['us'], 2) for key, v in d['roofline']['kernels'].items()}
    print(json.dumps(dict(lib='$n', round=$r, envs=int(envs), us_per_tick=d['gpu_ms_per_tick'] * 1e3, **k)))
" >> $OUT 2> /tmp/abl.err || { tail -5 /tmp/abl.err; exit 3; }
done; done
python3 - $OUT <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l)
    d[(j["envs"], j["lib"])].append((round(j["us_per_tick"], 1), j.get("acting"), j.get("critic_step"), j.get("actor_step")))
for k, v in sorted(d.items()): print(k, v)
PY
