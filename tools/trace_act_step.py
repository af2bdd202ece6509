"""Phase timeline of k_act_step32 (the self-play tick's fp32 actor forward +
env step + ring insert in one launch) from a -DSK_TRACE32 build:

    tools/build_variant.sh ab/trace32.so -DSK_TRACE32
    SK_LIB_PATH=$PWD/ab/trace32.so python tools/trace_act_step.py [--games 4096]

Microseconds from the first workgroup's first timestamp to each trace point,
first and last workgroup (s_memrealtime, 100 MHz)."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

POINTS = ["start", "step_loads_issued", "staged", "layer1", "layer2", "layer3", "actions_in_lds", "step_done"]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--games", default="4096,32768")
    p.add_argument("--noise", default="action")
    a = p.parse_args()
    from skillshot_learning_amd import learner
    from skillshot_learning_amd.actor_kernel import ActorKernel32
    from skillshot_learning_amd.vec_env import VecSkillshotGame
    torch.manual_seed(0)
    actor = learner.Actor().cuda()
    k = ActorKernel32(actor, seed=1)
    L = k.L
    L.sk_debug_trace32.argtypes = [ctypes.c_void_p]
    sd, asd = (0.5, 0.0) if a.noise == "param" else ((0.0, 0.15) if a.noise == "action" else (0.0, 0.0))
    for n in [int(x) for x in a.games.split(",")]:
        env = VecSkillshotGame(n, device="cuda", seed=3)
        ring = learner.ReplayRing(1 << 20, "cuda", seed=1)
        obs = env.observe()[0].clone()
        for _ in range(6):
            out = env.act_step(k, obs, noise_sd=sd, action_sd=asd, ring=ring)
            obs = out["obs_reset"].clone()
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (2 * 32 * 2))()
        assert L.sk_debug_trace32(buf) == 0
        t = np.frombuffer(buf, dtype=np.uint64).reshape(2, 32, 2).astype(np.float64)
        t0 = min(t[0, 0, 1], t[1, 0, 1])
        res = {}
        for wg in (0, 1):
            rt = t[wg, :len(POINTS), 1]
            res["first" if wg == 0 else "last"] = {nm: round(float((x - t0) / 100.0), 2) for nm, x in zip(POINTS, rt)}
        print(json.dumps({"kernel": "k_act_step32", "games": n, "noise": a.noise, **res}), flush=True)


if __name__ == "__main__":
    main()
