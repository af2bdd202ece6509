"""Throughput of the MFMA MLP kernels (sk_actor.hip, sk_critic.hip) against the
gfx950 bf16 dense MFMA peak and HBM, graph-replayed, timed with HIP events on
the launch stream.  One JSON line per (kernel, rows).

    python tools/bench_mlp_kernels.py [--rows 8192,131072,1048576] [--reps 200]
    python tools/bench_mlp_kernels.py --eager --only actor_noise --rows 131072 --reps 100   # for rocprofv3 --pmc

FLOP per row (2 x MACs): actor 72,192 (the noise
variant adds the variance-chain MFMAs on squared operands: 2x the layer-1/2
MACs); critic 72,448; target-Q = actor + critic.  Bytes per row: obs in 48,
actions in/out 8, Q out 4 (weights are read once per workgroup from L2).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK_TFLOPS = 2500.0   # bf16 dense MFMA, MI355X_MICROARCH.md
PEAK_GBS = 8000.0
ACTOR_FLOP = 2 * (12 * 256 + 256 * 128 + 128 * 2)
ACTOR_NOISE_FLOP = ACTOR_FLOP + 2 * (12 * 256 + 256 * 128)
CRITIC_FLOP = 2 * (12 * 256 + (256 + 2) * 128 + 128)
BWD_FLOP = 2 * (2 * 256 * 128 + 256 * 12)  # dW2, dH1, dW1 (the MFMA GEMMs of a backward)
CRITIC_GRAD_FLOP = CRITIC_FLOP + BWD_FLOP
ACTOR_GRAD_FLOP = ACTOR_FLOP + CRITIC_FLOP + BWD_FLOP


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", default="256,4096,8192,131072,1048576")
    p.add_argument("--reps", type=int, default=200)
    p.add_argument("--only", default="")
    p.add_argument("--eager", action="store_true", help="plain launches (rocprofv3 --pmc attribution)")
    a = p.parse_args()
    from skillshot_learning_amd import learner
    from skillshot_learning_amd.actor_kernel import ActorKernel
    from skillshot_learning_amd.critic_kernel import CriticKernel, TargetQKernel
    from skillshot_learning_amd.update_kernel import FusedUpdate

    torch.manual_seed(0)
    actor, critic = learner.Actor().cuda(), learner.Critic().cuda().eval()
    ak, ck, tk = ActorKernel(actor, seed=1), CriticKernel(critic), TargetQKernel(actor, critic)
    ddpg = learner.DDPG("cuda", seed=0, fused_update=True, precision="bf16")
    fu = ddpg._fused
    st = torch.cuda.Stream()
    for rows in [int(r) for r in a.rows.split(",")]:
        s = torch.rand(rows, 12, device="cuda")
        act = torch.rand(rows, 2, device="cuda") * 2 - 1
        y = torch.empty(rows, 2, device="cuda")
        q = torch.empty(rows, device="cuda")
        rw = torch.rand(rows, device="cuda")
        dn = torch.zeros(rows, device="cuda")
        cases = {
            "actor": (lambda: ak(s, 0.0, out=y), ACTOR_FLOP, 56),
            "actor_noise": (lambda: ak(s, 0.5, out=y), ACTOR_NOISE_FLOP, 56),
            "critic": (lambda: ck(s, act, out=q), CRITIC_FLOP, 60),
            "target_q": (lambda: tk(s, out=q), ACTOR_FLOP + CRITIC_FLOP, 52),
            "critic_grad": (lambda: fu.grads("critic", s, act, q), CRITIC_GRAD_FLOP, 60),
            "critic_grad_boot": (lambda: fu.grads("critic", s, act, None, None, s, rw, dn, 0.99),
                                 CRITIC_GRAD_FLOP + ACTOR_FLOP + CRITIC_FLOP, 116),
            "actor_grad": (lambda: fu.grads("actor", s), ACTOR_GRAD_FLOP, 48),
        }
        for name, (fn, flop, byts) in cases.items():
            if a.only and name != a.only:
                continue
            with torch.cuda.stream(st):
                fn()
                st.synchronize()
                if a.eager:
                    for _ in range(a.reps):
                        fn()
                    st.synchronize()
                    continue
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=st):
                    for _ in range(a.reps):
                        fn()
                g.replay()
                st.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                g.replay()
                e1.record(st)
                e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            tf = flop * rows / (us * 1e-6) / 1e12
            print(json.dumps({"kernel": name, "rows": rows, "us_per_launch": us, "tflops": tf,
                              "mfma_frac": tf / PEAK_TFLOPS, "gbs": byts * rows / (us * 1e-6) / 1e9,
                              "hbm_frac": byts * rows / (us * 1e-6) / 1e9 / PEAK_GBS,
                              "flop_per_row": flop}), flush=True)


if __name__ == "__main__":
    main()
