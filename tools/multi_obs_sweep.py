"""A/B: the full-contract multi-tick kernel (sk_env_step_multi_obs) per
games-per-GPU, ticks per launch, workgroup size, stagger, state port and
output-ring size; HIP events on the launch stream; one JSON line each.

    python tools/multi_obs_sweep.py [--envs 8192,65536] [--ticks 20,400] [--blocks 64,512] [--slabs 64]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def rate(n, T, block, stagger, pol, slabs, K=2000, prefetch=0):
    os.environ["SK_MULTI_PREFETCH"] = str(prefetch)
    os.environ["SK_MULTI_BLOCK"] = str(block)
    os.environ["SK_MULTI_STAGGER"] = str(stagger)
    os.environ["SK_MULTI_POLICY"] = str(pol)
    el, ev, env = bench.timed_multi_obs(torch.device("cuda", 0), n, 3, 0, 2000, K, 200, 400, slabs, per_launch=T)
    env.close()
    torch.cuda.empty_cache()
    us = ev * 1e3 / K
    return dict(envs=n, ticks_per_launch=T, block=block, prefetch=prefetch, stagger=stagger, policy=pol, out_slabs=slabs,
                us_per_tick=us, env_steps_per_s=n / (us * 1e-6), frac=297 * n / (us * 1e-6) / 8e12)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", default="65536")
    ap.add_argument("--ticks", default="20,400")
    ap.add_argument("--blocks", default="64,512")
    ap.add_argument("--staggers", default="0")
    ap.add_argument("--pols", default="1")
    ap.add_argument("--slabs", default="64")
    ap.add_argument("--prefetches", default="0", help="SK_MULTI_PREFETCH values")
    ap.add_argument("--passes", type=int, default=2)
    a = ap.parse_args()
    L = lambda s: [int(x) for x in s.split(",")]  # noqa: E731
    for p in range(a.passes):
        for n in L(a.envs):
            for T in L(a.ticks):
                for b in L(a.blocks):
                    for sg in L(a.staggers):
                        if sg and b != 512:
                            continue
                        for pol in L(a.pols):
                            for sl in L(a.slabs):
                                for pf in L(a.prefetches):
                                    r = rate(n, T, b, sg, pol, sl, prefetch=pf)
                                    print(json.dumps(dict(r, **{"pass": p})), flush=True)


if __name__ == "__main__":
    main()
