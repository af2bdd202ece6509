"""A/B: k_step_multi (T ticks per launch) against one graph-replayed k_step
launch per tick, per games-per-GPU and state port.  HIP events on the launch
stream; one JSON line per configuration.

    python tools/multi_sweep.py [--envs 8192,65536] [--ticks 1,5,20,100,400] [--pols 0,1]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def multi_rate(n, T, pol, split=-1, stagger=0, block=-1, fast=0, early=-1, K=2000, ring=400, seed=0, prefetch=0,
               pack=-1):
    os.environ["SK_MULTI_PREFETCH"] = str(prefetch)
    os.environ["SK_MULTI_PACK"] = str(pack)
    os.environ["SK_MULTI_FAST"] = str(fast)
    os.environ["SK_MULTI_EARLY"] = str(early)
    os.environ["SK_MULTI_BLOCK"] = str(block)
    os.environ["SK_MULTI_POLICY"] = str(pol)
    os.environ["SK_MULTI_SPLIT"] = str(split)
    os.environ["SK_MULTI_STAGGER"] = str(stagger)
    from skillshot_learning_amd import VecSkillshotGame
    dev = torch.device("cuda", 0)
    env = VecSkillshotGame(n, device=dev, seed=seed, tick_limit=2000, random_positions=True)
    st = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(st):
        env.reset(random_positions=True)
        acts = env.gen_random_actions(ring)
    done = torch.empty(n, dtype=torch.uint8, device=dev)
    sp, ap, dp = ctypes.c_void_p(st.cuda_stream), ctypes.c_void_p(acts.data_ptr()), ctypes.c_void_p(done.data_ptr())
    launches = max(1, K // T)
    slab = 0

    def go(m):
        nonlocal slab
        for _ in range(m):
            env.step_multi_raw(ap, ring, slab, T, dp, None, 0, stream=sp)
            slab = (slab + T) % ring

    go(3)
    st.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        e0.record()
    go(launches)
    with torch.cuda.stream(st):
        e1.record()
    st.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (launches * T)
    env.close()
    return dict(kind="multi", envs=n, ring=ring, prefetch=prefetch, pack=pack, ticks_per_launch=T, policy=pol, split=split, stagger=stagger, block=block, fast=fast, early=early, us_per_tick=us,
                env_steps_per_s=n / (us * 1e-6), frac=193 * n / (us * 1e-6) / 8e12)


def graph_rate(n, K=2000, ring=400, seed=0):
    el, ev, env = bench.timed_ticks(torch.device("cuda", 0), n, seed, 0, 2000, K, 200, ring, 400, 1)
    env.close()
    us = ev * 1e3 / K
    return dict(kind="k_step graph", envs=n, us_per_tick=us, env_steps_per_s=n / (us * 1e-6),
                frac=193 * n / (us * 1e-6) / 8e12)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", default="8192,65536")
    p.add_argument("--ticks", default="1,5,20,100,400")
    p.add_argument("--pols", default="0,1")
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--splits", default="-1")
    p.add_argument("--staggers", default="0")
    p.add_argument("--blocks", default="-1")
    p.add_argument("--fasts", default="0")
    p.add_argument("--earlys", default="-1")
    p.add_argument("--rings", default="400", help="action slabs in the ring (400: larger than the Infinity Cache)")
    p.add_argument("--prefetches", default="0", help="SK_MULTI_PREFETCH values (k_step_multi's prefetch wave)")
    p.add_argument("--packs", default="-1", help="SK_MULTI_PACK values (-1 auto, 0 88-B form, 1 packed form)")
    p.add_argument("--no-graph", action="store_true")
    a = p.parse_args()
    torch.cuda.set_device(0)
    for rep in range(a.reps):
        for n in [int(x) for x in a.envs.split(",")]:
            if not a.no_graph:
                print(json.dumps(dict(graph_rate(n), rep=rep)), flush=True)
            for pol in [int(x) for x in a.pols.split(",")]:
                for sp in [int(x) for x in a.splits.split(",")]:
                    for T in [int(x) for x in a.ticks.split(",")]:
                        for sg in [int(x) for x in a.staggers.split(",")]:
                            for bk in [int(x) for x in a.blocks.split(",")]:
                                for fa in [int(x) for x in a.fasts.split(",")]:
                                    for ea in [int(x) for x in a.earlys.split(",")]:
                                        for rg in [int(x) for x in a.rings.split(",")]:
                                            for pf in [int(x) for x in a.prefetches.split(",")]:
                                                for pk in [int(x) for x in a.packs.split(",")]:
                                                    r = multi_rate(n, T, pol, sp, sg, bk, fa, ea, ring=rg, prefetch=pf,
                                                                   pack=pk)
                                                    print(json.dumps(dict(r, rep=rep)), flush=True)


if __name__ == "__main__":
    main()
