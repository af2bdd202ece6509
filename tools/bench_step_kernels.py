"""Device time of the one-tick step kernels the learner's acting uses, per
game count: sk_env_step with obs + reward (k_step_split), sk_env_step_insert
(the same + the replay ring insert), and the fp32 actor forward beside them
(sk_actor_forward_f32 with parameter noise).  HIP events around one replay
of a hipGraph of --iters launches.

    python tools/bench_step_kernels.py [--games 4096,65536] [--iters 40]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, st, iters):
    with torch.cuda.stream(st):
        for _ in range(3):
            fn()
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st, capture_error_mode="thread_local"):
        for _ in range(iters):
            fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):  # replay() launches on the current stream
        g.replay()
        e0.record(st)
        g.replay()
        e1.record(st)
    st.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--games", default="4096,65536")
    p.add_argument("--iters", type=int, default=40)
    a = p.parse_args()
    from skillshot_learning_amd import learner
    from skillshot_learning_amd.actor_kernel import ActorKernel32
    from skillshot_learning_amd.vec_env import VecSkillshotGame
    torch.manual_seed(0)
    actor = learner.Actor().cuda()
    k = ActorKernel32(actor, seed=1)
    st = torch.cuda.Stream()
    for n in [int(x) for x in a.games.split(",")]:
        env = VecSkillshotGame(n, device="cuda", seed=3)
        ring = learner.ReplayRing(1 << 22, "cuda", seed=1)
        with torch.cuda.stream(st):
            obs = env.observe()[0].clone()
            acts = torch.rand((2, n, 2), device="cuda") * 2 - 1
            outbuf = dict(obs=env.new_obs(), reward=torch.empty((2, n), device="cuda"),
                          done=torch.empty(n, dtype=torch.uint8, device="cuda"),
                          winner=torch.empty(n, dtype=torch.uint8, device="cuda"), obs_reset=env.new_obs())
            a_out = torch.empty((2 * n, 2), device="cuda")
        st.synchronize()
        res = dict(games=n)
        res["step_obs_reward_us"] = timed(
            lambda: env.step(acts, obs=True, reward="looking", auto_reset=True, out=outbuf), st, a.iters)
        res["step_insert_us"] = timed(lambda: env.step_insert(acts, obs, ring, out=outbuf), st, a.iters)
        res["actor_fwd_param_us"] = timed(lambda: k(obs.reshape(-1, 12), noise_sd=0.5, out=a_out), st, a.iters)
        res["act_step_param_us"] = timed(lambda: env.act_step(k, obs, noise_sd=0.5, ring=ring, out=outbuf), st,
                                         a.iters)
        print(json.dumps(res), flush=True)
        env.close()


if __name__ == "__main__":
    main()
