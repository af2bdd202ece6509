"""Learner-loop diagnostics: (1) episode counters against a direct sum of the
step's done flags, with action statistics of the initial policy; (2) host cost
of replaying a captured graph per kernel node."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from skillshot_learning_amd.learner import SkillshotLearner, STATE_DIM, ACTION_DIM  # noqa: E402

L = SkillshotLearner(n_envs=4096, seed=0, tick_limit=2000, replay_capacity=1 << 18)
g = L.game_environment
g.clear_counters()
obs = L.prepare_states()
done_sum = torch.zeros((), dtype=torch.int64, device="cuda")
amax = torch.zeros((), device="cuda")
for t in range(600):
    act = L.model_act(obs)
    out = L.do_actions(act, reset_obs=True)
    done_sum += out["done"].long().sum()
    amax = torch.maximum(amax, act.abs().max())
    obs = out["obs_reset"]
torch.cuda.synchronize()
print(json.dumps(dict(ticks=600, done_flags=int(done_sum), counters=g.counters(), max_abs_action=float(amax),
                      mean_abs_action=float(act.abs().mean()))))

# graph replay host cost vs node count
x = torch.zeros(1024, device="cuda")
for nodes in (10, 100, 400):
    s = torch.cuda.Stream()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1)
    torch.cuda.synchronize()
    with torch.cuda.graph(gr, stream=s):
        for _ in range(nodes):
            x.add_(1)
    torch.cuda.synchronize()
    for _ in range(5):
        gr.replay()
    torch.cuda.synchronize()
    reps = 50
    t0 = time.perf_counter()
    for _ in range(reps):
        gr.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(json.dumps(dict(nodes=nodes, host_us_per_replay=(t1 - t0) / reps * 1e6,
                          host_us_per_node=(t1 - t0) / reps / nodes * 1e6,
                          wall_us_per_replay=(t2 - t0) / reps * 1e6)))
