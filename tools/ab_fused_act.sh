cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04x
for r in 1 2; do for f in 1 0; do
SK_FUSED_ACT=$f timeout -k 10 200 python3 -c "
import bench, json
for cfg in ['65536:param_noise', '4096:action_noise']:
    envs, ex = cfg.split(':')
    d = bench.learner_rate(int(envs), 1, 0, 200, batch=256, exploration=ex, precision='fp32')
    k = {key: round(v['us'], 2) for key, v in d['roofline']['kernels'].items()}
    print(json.dumps(dict(fused=$f, round=$r, envs=int(envs), us_per_tick=d['gpu_ms_per_tick'] * 1e3, **k)))
" >> gpurun_out/r04x/fused_ab.jsonl || exit 3
done; done
timeout -k 10 200 python3 tools/bench_actor_fwd.py --rows 8192,131072 --precisions fp32 > gpurun_out/r04x/actor_fwd.jsonl
cat gpurun_out/r04x/fused_ab.jsonl gpurun_out/r04x/actor_fwd.jsonl
