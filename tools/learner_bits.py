"""Dump the nets after a fixed learner run, for bit-for-bit A/Bs of library
builds whose arithmetic must not change (summation-order-preserving kernel
rewrites):

    SK_LIB_PATH=old.so python tools/learner_bits.py --out /tmp/a.npz
    SK_LIB_PATH=new.so python tools/learner_bits.py --out /tmp/b.npz
    python tools/learner_bits.py --compare /tmp/a.npz /tmp/b.npz

Config 3's shape at a smaller size: 4,096 games, batch 256, fp32, action
noise, the replay-rule tick graph-replayed (critic + actor steps with target
nets, Adam, soft updates), then models_fit on a played epoch (the resident
fit and the three-launch steps) when --fit is given."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(a):
    from skillshot_learning_amd.learner import SkillshotLearner
    L = SkillshotLearner(n_envs=a.envs, device="cuda", seed=11, exploration=a.exploration, gamma=0.9, tau=0.05,
                         replay_capacity=1 << 16, precision="fp32")
    tg = L.tick_graph(batch=a.batch, ticks_per_graph=2, warmup=2)
    tg.run(a.replays)
    torch.cuda.synchronize()
    out = {}
    for name, m in (("actor", L.model_actor), ("critic", L.model_critic)):
        out[name] = torch.cat([p.detach().flatten() for p in m.parameters()]).cpu().numpy()
    fu = L.ddpg._fused
    for k in ("ta", "tc"):
        out[k] = getattr(fu, k).detach().cpu().numpy()
    out["ring"] = L.replay.buf.detach().cpu().numpy()
    np.savez(a.out, **out)
    print("wrote", a.out, {k: v.shape for k, v in out.items()})


def compare(fa, fb):
    A, B = np.load(fa), np.load(fb)
    ok = True
    for k in A.files:
        same = np.array_equal(A[k].view(np.uint8), B[k].view(np.uint8))
        diff = float(np.abs(A[k].astype(np.float64) - B[k].astype(np.float64)).max())
        print(k, "bit-identical" if same else f"DIFFERS (max abs {diff:.3g})")
        ok &= same
    sys.exit(0 if ok else 1)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--out", default="/tmp/learner_bits.npz")
    p.add_argument("--envs", type=int, default=4096)
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--replays", type=int, default=20)
    p.add_argument("--exploration", default="action_noise")
    p.add_argument("--compare", nargs=2)
    a = p.parse_args()
    if a.compare:
        compare(*a.compare)
    else:
        run(a)


if __name__ == "__main__":
    main()
