#!/bin/bash
# Alternating A/B of prebuilt library variants (ab_run/*.so, SK_LIB_PATH) on
# the reference rule's episode collection (bench.reference_rule_rate:
# sk_env_act_episode at 65,536 games, one launch):
#   PASSES=2 bash tools/ab_libs_episode.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
OUT=gpurun_out/${1:-ab_libs_episode}.jsonl; : > $OUT
for r in $(seq ${PASSES:-2}); do for f in ab_run/*.so; do n=$(basename $f .so)
  SK_LIB_PATH=$PWD/$f timeout -k 10 300 python3 -c "
import bench, json
d = bench.reference_rule_rate(${ENVS:-65536}, fit_chunks=2)
c = d['collection']
print(json.dumps(dict(lib='$n', round=$r, envs=d['envs'], ticks=d['episode_ticks_max'], gpu_s=c['gpu_s'],
                      us_per_tick=c['gpu_us_per_tick'], fit_us_per_step=d['fit']['us_per_minibatch_step'])))
" >> $OUT 2> /tmp/abe.err || { tail -5 /tmp/abe.err; exit 3; }
done; done
cat $OUT
