"""models_fit's per-minibatch-step time (the reference rule's fit,
SkillshotLearner.py:419-443): the resident critic and
actor passes (sk_fit_critic_f32, sk_fit_actor_f32) per workgroup count
(SK_FIT_P) and placement (SK_FIT_XCD), against the
three-launch steps replayed as captured chunks of 64 (the round-4 path);
HIP events, one JSON line per configuration.

    python tools/bench_fit.py [--steps 4096] [--reps 3]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=4096)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--resident-only", action="store_true", help="skip the three-launch chunks (PMC passes)")
    a = p.parse_args()
    from skillshot_learning_amd import learner
    dev = torch.device("cuda", 0)
    n = a.steps
    g = torch.Generator(device=dev).manual_seed(1)
    S = torch.rand(16 * n, 12, device=dev, generator=g)
    A = torch.rand(16 * n, 2, device=dev, generator=g) * 2 - 1
    R = torch.randn(16 * n, device=dev, generator=g)
    d = learner.DDPG("cuda", seed=0, fused_update=True, precision="fp32")
    fu = d._fused
    fu.soft_update_in_adam = False
    fu.FIT_STEPS_PER_LAUNCH = n
    st = torch.cuda.current_stream(dev)

    def timed(fn, steps):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / steps

    for rep in range(a.reps):
        cfgs = os.environ.get("BENCH_FIT_CFG", "16:0,16:1,8:1")
        for P, xcd in (c.split(":") for c in cfgs.split(",")):
            os.environ["SK_FIT_P"], os.environ["SK_FIT_XCD"] = P, xcd
            us = timed(lambda: fu.fit_critic(S, A, R), n)
            fu.fit_check()
            print(json.dumps(dict(kind="resident critic", P=int(P), one_xcd=xcd == "1", steps=n,
                                  us_per_step=round(us, 3), rep=rep)), flush=True)
            us = timed(lambda: fu.fit_actor(S), n)
            fu.fit_check()
            print(json.dumps(dict(kind="resident actor", P=int(P), one_xcd=xcd == "1", steps=n,
                                  us_per_step=round(us, 3), rep=rep)), flush=True)
        if a.resident_only:
            continue
        M = d.FIT_CHUNK
        chunks = n // M - 1
        for critic in (True, False):
            us = timed(lambda: d._fit_chunks(S, A, R, 16, M, chunks, critic=critic), chunks * M)
            print(json.dumps(dict(kind="three-launch " + ("critic" if critic else "actor"),
                                  steps=chunks * M, us_per_step=round(us, 3), rep=rep)), flush=True)


if __name__ == "__main__":
    main()
