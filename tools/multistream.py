"""Experiment: the 65,536-game step as S independent shards on S HIP streams.

Games never interact, so shard s (games [s*n/S, (s+1)*n/S), keyed by global
id exactly like the multi-GPU split) can run its tick chain on its own stream;
the S chains overlap each other's dependent-launch gaps.  Prints one JSON
line per S with the wall-clock env-steps/s over K ticks of all games.

    python tools/multistream.py [--envs 65536] [--shards 1,2,4,8] [--steps 4000]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(n, S, K, G, ring, seed=0):
    from skillshot_learning_amd import VecSkillshotGame
    m = n // S
    envs, streams, graphs, acts, dones = [], [], [], [], []
    for s in range(S):
        st = torch.cuda.Stream()
        e = VecSkillshotGame(m, seed=seed, env_offset=s * m, tick_limit=2000, random_positions=True)
        with torch.cuda.stream(st):
            e.reset(random_positions=True)
            a = e.gen_random_actions(ring)
            d = torch.empty(m, dtype=torch.uint8, device="cuda")
        envs.append(e), streams.append(st), acts.append(a), dones.append(d)
    torch.cuda.synchronize()
    for s in range(S):
        e, st, a, d = envs[s], streams[s], acts[s], dones[s]
        slab = 2 * m * 2 * 4
        sp = ctypes.c_void_p(st.cuda_stream)

        def launch(t, e=e, a=a, d=d, sp=sp, slab=slab):
            e.step_raw(ctypes.c_void_p(a.data_ptr() + (t % ring) * slab), ctypes.c_void_p(d.data_ptr()), stream=sp)

        with torch.cuda.stream(st):
            for t in range(4):
                launch(t)
        st.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for t in range(G):
                launch(t)
        st.synchronize()
        graphs.append(g)

    def go(reps):
        for _ in range(reps):
            for s in range(S):
                with torch.cuda.stream(streams[s]):
                    graphs[s].replay()

    go(2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    go(K // G)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    steps = (K // G) * G
    res = dict(envs=n, shards=S, ticks=steps, us_per_tick=el * 1e6 / steps, env_steps_per_s=n * steps / el,
               frac_193B=n * steps * 193 / el / 8e12,
               dones=sum(e.counters()["dones"] for e in envs))
    for e in envs:
        e.close()
    return res


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=65536)
    p.add_argument("--shards", default="1,2,4,8")
    p.add_argument("--steps", type=int, default=4000)
    p.add_argument("--graph-len", type=int, default=400)
    p.add_argument("--ring", type=int, default=400)
    a = p.parse_args()
    for S in [int(x) for x in a.shards.split(",")]:
        print(json.dumps(run(a.envs, S, a.steps, a.graph_len, a.ring)), flush=True)


if __name__ == "__main__":
    main()
