#!/bin/bash
# A/B of ab_run/*.so on the standalone fp32 actor forward (bench_actor_fwd.py,
# 131,072 rows) and on config 5's tick with the fused (SK_FUSED_ACT=1) and
# the unfused acting (actor forward launch + sk_env_step_insert):
#   PASSES=2 bash tools/ab_fwd_waves.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
OUT=gpurun_out/${1:-ab_fwd_waves}.jsonl; : > $OUT
for r in $(seq ${PASSES:-2}); do for f in ab_run/*.so; do n=$(basename $f .so)
  SK_LIB_PATH=$PWD/$f timeout -k 10 120 python3 tools/bench_actor_fwd.py --rows 131072 --precisions fp32 \
    | sed "s/^{/{\"lib\": \"$n\", \"round\": $r, /" >> $OUT || exit 3
  for fa in 1 0; do
    SK_LIB_PATH=$PWD/$f SK_FUSED_ACT=$fa timeout -k 10 200 python3 -c "
import bench, json
d = bench.learner_rate(65536, 1, 0, 200, batch=256, exploration='param_noise', precision='fp32')
k = {key: round(v['us'], 2) for key, v in d['roofline']['kernels'].items()}
print(json.dumps(dict(lib='$n', round=$r, fused_act=$fa, us_per_tick=d['gpu_ms_per_tick'] * 1e3, **k)))
" >> $OUT || exit 3
  done
done; done
cat $OUT
