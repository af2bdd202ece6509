cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out/knobs.jsonl; : > $O
for kv in "NONE=1" "DEBUG_CLR_SKIP_RELEASE_SCOPE=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "HIP_FORCE_DEV_KERNARG=0" "HIP_FORCE_DEV_KERNARG=1" "DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0"; do
  env $kv timeout -k 10 120 python tools/sweep.py --variants empty,0 --envs 65536 --steps 2000 > gpurun_out/k.jsonl 2>gpurun_out/k.err || { echo "fail $kv"; tail -3 gpurun_out/k.err; break; }
  sed "s/^/{\"knob\": \"$kv\", \"r\": /; s/$/}/" gpurun_out/k.jsonl >> $O
done
cat $O
