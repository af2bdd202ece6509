#!/bin/bash
# Short timed regions (driver's --steps 20): does the host's wait mode account
# for the wall-vs-event gap?  Each variant in its own process, own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
O=gpurun_out/wait_knobs.jsonl; : > $O
for v in "" "ROC_ACTIVE_WAIT_TIMEOUT=0" "ROC_ACTIVE_WAIT_TIMEOUT=1000" "ROC_ACTIVE_WAIT_TIMEOUT=100000" "SPIN" "ROC_CPU_WAIT_FOR_SIGNAL=0"; do
  if [ "$v" = SPIN ]; then
    timeout -k 10 120 python tools/short_run_overhead.py --spin >> $O 2>/dev/null || exit $?
  else
    timeout -k 10 120 env $v python tools/short_run_overhead.py >> $O 2>/dev/null || exit $?
  fi
done
cat $O
