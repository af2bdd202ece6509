"""Why does the GPU learner see no episode ends?  Drive the GPU env with the
initial actor through (a) the fused actor kernel, (b) the torch
local-reparameterisation forward, and report state statistics."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from skillshot_learning_amd.learner import SkillshotLearner  # noqa: E402

for use_kernel in (True, False):
    L = SkillshotLearner(n_envs=4096, seed=0, tick_limit=2000, replay_capacity=1 << 10,
                         actor_kernel=use_kernel)
    g = L.game_environment
    obs = L.prepare_states()
    o0 = obs.clone()
    look = []
    for t in range(600):
        act = L.model_act(obs)
        look.append(float(act[..., 1].abs().mean()))
        out = L.do_actions(act, reset_obs=True)
        obs = out["obs_reset"]
    torch.cuda.synchronize()
    sd = g.state_dict()
    rot = sd["rot"]
    a_det = L.model_act(o0, mode="deterministic")
    ref = L.model_actor(o0.reshape(-1, 12)).reshape(2, -1, 2)
    print(json.dumps(dict(kernel=use_kernel, counters=g.counters(), rot_min=float(rot.min()), rot_max=float(rot.max()),
                          mean_abs_look=sum(look) / len(look), ticks=int(sd["misc"][:, 0].max()),
                          obs0_row0=o0[0, 0].tolist(), act_det_row0=a_det[0, 0].tolist(),
                          torch_det_row0=ref[0, 0].tolist(),
                          det_maxdiff=float((a_det - ref).abs().max()))), flush=True)
