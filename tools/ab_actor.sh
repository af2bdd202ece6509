#!/bin/bash
# Alternating A/B (3 passes) of prebuilt ab/*.so on the actor forward
# (tools/bench_actor_fwd.py: fp32 / bf16, with and without parameter noise).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-ab_actor}.jsonl; : > $OUT
for r in 1 2 3; do for f in ab/*.so; do n=$(basename $f .so)
  SK_LIB_PATH=$PWD/$f timeout -k 10 200 python tools/bench_actor_fwd.py --rows ${ROWS:-8192,131072} > /tmp/aa.jsonl 2> /tmp/aa_err.txt || { tail -5 /tmp/aa_err.txt; exit 3; }
  sed "s/^/{\"lib\": \"$n\", \"round\": $r, \"r\": /; s/$/}/" /tmp/aa.jsonl >> $OUT
done; done
python3 - $OUT <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l); r = j["r"]; d[(j["lib"], r["precision"], r["rows"], r["param_noise"], r.get("action_noise", 0.0))].append(r["us"])
for k, v in sorted(d.items()): print(k, [round(x, 2) for x in v])
PY
