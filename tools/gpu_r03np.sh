#!/bin/bash
# fp32 parameter noise in pair form (Philox 7 / 10 rounds) vs the previous
# normals4 form: the fp32 actor tests (KS), then the noisy fp32 forward at
# 8,192 / 131,072 rows and the config-5 / config-3-param-noise ticks,
# alternating library variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
O=gpurun_out/r03np; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_learn32_gpu.py tests/test_replay_gpu.py tests/test_actor_gpu.py tests/test_config3_gpu.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; grep -E "^(FAILED|ERROR)" $O/pytest.txt; tail -2 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
: > $O/ab.jsonl
for rep in 1 2; do
  for v in prev pair10 pair7; do
    SK_LIB_PATH=$PWD/ab/$v.so timeout -k 10 120 python -u tools/bench_actor_fwd.py --rows 8192,131072 --precisions fp32 2>> $O/err.txt | grep '"param_noise": 0.5' | sed "s/^{/{\"lib\": \"$v\", \"rep\": $rep, /" >> $O/ab.jsonl || { tail -20 $O/err.txt; exit 1; }
    SK_LIB_PATH=$PWD/ab/$v.so timeout -k 10 200 python -u -c "
import json, bench
for envs in (65536, 4096):
    r = bench.learner_rate(envs, 1, 0, 400, batch=256, exploration='param_noise', precision='fp32')
    print(json.dumps(dict(lib='$v', rep=$rep, envs=envs, tick_mode=r['tick_mode'], us_per_tick=round(r['ms_per_tick'] * 1e3, 2))), flush=True)
" >> $O/ab.jsonl 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
cat $O/ab.jsonl
