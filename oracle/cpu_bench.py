"""Timed CPU run of the oracle step (TEST INFRASTRUCTURE: the cpu_baseline leg
of bench.py, one process per core).  The same workload as the GPU headline:
random-policy actions pre-generated (untimed), fused step with auto-reset.

    python -m oracle.cpu_bench --envs 4096 --env-offset 0 --seconds 10
prints one JSON line {"envs", "ticks", "seconds", "env_steps_per_s"}.

run_python: SURVEY.md §8(d) config 1 on the pure-Python restatement
(oracle/pyoracle.py) — one game, random.Random(seed).uniform(-1, 1) actions in
do_actions order, game_tick, random reset on done or at 2000 ticks — the
procedure BASELINE.md times the reference with, so the two rates relate by
the ratio tools/ref_ratio.py measures where the reference is importable.
"""
import random
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


def run_python(seconds, seed=0, tick_limit=2000):
    from oracle.pyoracle import Game
    rng = random.Random(seed)
    g = Game()

    def reset():
        g.__init__()
        g.x = [rng.randrange(25, 225), rng.randrange(25, 225)]
        g.y = [rng.randrange(25, 225), rng.randrange(25, 225)]

    reset()
    steps = 0
    t0 = time.perf_counter()
    while True:
        for _ in range(1000):
            for p in (0, 1):
                g.move_direction(p, rng.uniform(-1, 1))
                g.move_look(p, rng.uniform(-1, 1))
                g.shoot(p)
            g.game_tick()
            if not g.live or g.ticks >= tick_limit:
                reset()
        steps += 1000
        el = time.perf_counter() - t0
        if el >= seconds:
            return dict(envs=1, ticks=steps, seconds=el, env_steps_per_s=steps / el)


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=4096)
    p.add_argument("--env-offset", type=int, default=0)
    p.add_argument("--seconds", type=float, default=10.0)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--tick-limit", type=int, default=2000)
    p.add_argument("--python", action="store_true", help="config 1 on the pure-Python restatement")
    a = p.parse_args()
    r = run_python(a.seconds, a.seed, a.tick_limit) if a.python else run(a.envs, a.seconds, a.env_offset, a.seed,
                                                                         a.tick_limit)
    print(json.dumps(r), flush=True)
