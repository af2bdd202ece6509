"""Timed CPU run of the oracle step (TEST INFRASTRUCTURE: the cpu_baseline leg
of bench.py, one process per core).  The same workload as the GPU headline:
random-policy actions pre-generated (untimed), fused step with auto-reset.

    python -m oracle.cpu_bench --envs 4096 --env-offset 0 --seconds 10
prints one JSON line {"envs", "ticks", "seconds", "env_steps_per_s"}.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import oracle  # noqa: E402


def run(n, seconds, env_offset=0, seed=0, tick_limit=2000, chunk=8):
    s = oracle.OracleState(n, seed=seed, env_offset=env_offset)
    s.reset(random_positions=True)
    acts = s.gen_random_actions(chunk)
    steps = 0
    t0 = time.perf_counter()
    while True:
        for t in range(chunk):
            s.step(acts[t], tick_limit=tick_limit, auto_reset=True, random_positions=True, want_obs=False)
        steps += chunk
        el = time.perf_counter() - t0
        if el >= seconds:
            return dict(envs=n, ticks=steps, seconds=el, env_steps_per_s=n * steps / el)


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=4096)
    p.add_argument("--env-offset", type=int, default=0)
    p.add_argument("--seconds", type=float, default=10.0)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--tick-limit", type=int, default=2000)
    a = p.parse_args()
    print(json.dumps(run(a.envs, a.seconds, a.env_offset, a.seed, a.tick_limit)), flush=True)
