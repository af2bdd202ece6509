"""Resident critic pass vs the three-launch chain over long passes: max
parameter difference after n steps for one launch (the Adam step-size table
refilled in-launch past 2,048 steps) and for launches cut every 2,048 steps
(no refill), to tell a refill fault from chaotic divergence of two fp32
summation orders.   python tools/diag_fit_long.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from skillshot_learning_amd import learner
    dev = torch.device("cuda", 0)

    def rows(n, seed):
        g = torch.Generator(device=dev).manual_seed(seed)
        s = torch.rand(16 * n, 12, device=dev, generator=g) * torch.tensor(
            [1, 1, 1, 1, 9.8, 1, 1, 1, 1, 9.8, 1, 1.0], device=dev)
        return s, torch.rand(16 * n, 2, device=dev, generator=g) * 2 - 1, torch.randn(16 * n, device=dev,
                                                                                       generator=g) * 0.5

    for n in (256, 1024, 2040, 2100, 2600):
        s, a, y = rows(n, 13)
        out = dict(n=n)
        ref = learner.DDPG("cuda", seed=6, fused_update=True, precision="fp32")
        trace = []
        for k in range(n):
            ref.critic_step(s[16 * k:16 * k + 16], a[16 * k:16 * k + 16], y[16 * k:16 * k + 16])
        torch.cuda.synchronize()
        for per in (4096, 2048, 512):
            d = learner.DDPG("cuda", seed=6, fused_update=True, precision="fp32")
            d._fused.FIT_STEPS_PER_LAUNCH = per
            d._fused.fit_critic(s, a, y)
            d._fused.fit_check()
            torch.cuda.synchronize()
            out[f"err_per{per}"] = (d._fused.fc - ref._fused.fc).abs().max().item()
            out[f"steps_eq_per{per}"] = bool(torch.equal(d._fused.sc.steps, ref._fused.sc.steps))
        # two resident runs with different launch cuts against each other
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
