#!/bin/bash
# Alternating A/B of prebuilt libraries (LIBS, default ab_run/old.so ab_run/new.so)
# on the headline leg at the driver's K = 20 and at K = 4,000: three passes,
# one JSON line per run (wall us/step, event us/step, frac) -> gpurun_out/ab_k20.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
LIBS=${LIBS:-"ab_run/old.so ab_run/new.so"}
for r in 1 2 3; do for f in $LIBS; do n=$(basename $f .so)
  for k in ${KS:-20 4000}; do w=$([ $k = 20 ] && echo 5 || echo 400)
    SK_LIB_PATH=$PWD/$f timeout -k 10 200 python bench.py --steps $k --warmup $w --no-learner --no-cpu-baseline \
      --no-large --no-full --no-rollout --no-variants > gpurun_out/abk_${n}_${k}_${r}.json 2>gpurun_out/abk_err.txt || exit 3
    python -c "import json; d=json.loads(open('gpurun_out/abk_${n}_${k}_${r}.json').read().strip().splitlines()[-1]); print(json.dumps({'lib':'$n','K':$k,'pass':$r,'wall_us':round(d['ms_per_step']*1e3,4),'event_us':round(d['config']['event_ms_per_step']*1e3,4),'frac':d['roofline']['frac'],'episodes':d.get('episodes')}))" | tee -a gpurun_out/ab_k20.jsonl
  done
done; done
