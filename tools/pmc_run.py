"""Eager k_step (or, --multi T, k_step_multi) launches for rocprofv3 --pmc passes (graph replay is avoided so
every dispatch is attributed).  Same workload as bench.py (random policy,
pre-generated actions ring, done output, random auto-reset).

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT -o pmc \
        -- python3 tools/pmc_run.py --envs 65536 --launches 300
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=65536)
    p.add_argument("--launches", type=int, default=300)
    p.add_argument("--ring", type=int, default=300)
    p.add_argument("--obs", action="store_true")
    p.add_argument("--multi", type=int, default=0, help="k_step_multi launches of this many ticks instead")
    p.add_argument("--multi-obs", type=int, default=0,
                   help="sk_env_step_multi_obs launches (full contract) of this many ticks instead")
    p.add_argument("--out-slabs", type=int, default=64, help="--multi-obs: output ring slabs")
    a = p.parse_args()
    from skillshot_learning_amd import VecSkillshotGame
    n = a.envs
    env = VecSkillshotGame(n, seed=0, tick_limit=2000)
    env.reset(random_positions=True)
    acts = env.gen_random_actions(a.ring)
    done = torch.empty(n, dtype=torch.uint8, device="cuda")
    o = torch.empty((2, n, 12), dtype=torch.float32, device="cuda") if a.obs else None
    r = torch.empty((2, n), dtype=torch.float32, device="cuda") if a.obs else None
    torch.cuda.synchronize()
    if a.multi_obs:
        S = a.out_slabs
        out = dict(obs=torch.empty((S, 2, n, 12), dtype=torch.float32, device="cuda"),
                   reward=torch.empty((S, 2, n), dtype=torch.float32, device="cuda"),
                   done=torch.empty((S, n), dtype=torch.uint8, device="cuda"), winner=None)
        slab, so = 0, 0
        for _ in range(a.launches):
            env.step_multi_obs(acts, n_ticks=a.multi_obs, slab0=slab, out_slabs=S, out0=so, out=out)
            slab = (slab + a.multi_obs) % a.ring
            so = (so + a.multi_obs) % S
        torch.cuda.synchronize()
        print("multi_obs launches", a.launches, "x", a.multi_obs, "ticks, envs", n)
        return
    if a.multi:
        slab = 0
        for _ in range(a.launches):
            env.step_multi_raw(ctypes.c_void_p(acts.data_ptr()), a.ring, slab, a.multi, ctypes.c_void_p(done.data_ptr()))
            slab = (slab + a.multi) % a.ring
        torch.cuda.synchronize()
        print("multi launches", a.launches, "x", a.multi, "ticks, envs", n)
        return
    for t in range(a.launches):
        env.step_raw(ctypes.c_void_p(acts.data_ptr() + (t % a.ring) * 16 * n), ctypes.c_void_p(done.data_ptr()),
                     obs_ptr=None if o is None else ctypes.c_void_p(o.data_ptr()),
                     reward_ptr=None if r is None else ctypes.c_void_p(r.data_ptr()))
    torch.cuda.synchronize()
    print("launches", a.launches, "envs", n)


if __name__ == "__main__":
    main()
