"""Eager acting launches of the config-5 tick (sk_env_act_step ->
k_act_step32<true>: the fp32 actor with parameter noise sd 0.5 on split-bf16
MFMAs + env step + obs / reward + ring insert, 65,536 games) and of config 3's
action-noise form, for rocprofv3 --pmc passes (tools/pmc_act_step.sh).

    rocprofv3 --pmc SQ_INSTS_VALU ... --output-format csv -d OUT -o pmc \
        -- python3 tools/pmc_act_step.py --games 65536 --launches 30
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--games", type=int, default=65536)
    p.add_argument("--launches", type=int, default=30)
    p.add_argument("--noise", default="param", choices=["param", "action"])
    a = p.parse_args()
    from skillshot_learning_amd import learner
    from skillshot_learning_amd.actor_kernel import ActorKernel32
    from skillshot_learning_amd.vec_env import VecSkillshotGame
    torch.manual_seed(0)
    actor = learner.Actor().cuda()
    k = ActorKernel32(actor, seed=1)
    sd, asd = (0.5, 0.0) if a.noise == "param" else (0.0, 0.15)
    env = VecSkillshotGame(a.games, device="cuda", seed=3)
    ring = learner.ReplayRing(1 << 20, "cuda", seed=1)
    obs = env.observe()[0].clone()
    for _ in range(a.launches):
        out = env.act_step(k, obs, noise_sd=sd, action_sd=asd, ring=ring)
        obs = out["obs_reset"]
    torch.cuda.synchronize()
    print("act_step launches", a.launches, "games", a.games, "noise", a.noise)


if __name__ == "__main__":
    main()
