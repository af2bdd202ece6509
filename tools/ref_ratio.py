"""Speed of the pure-Python restatement (oracle/pyoracle.py) relative to the
reference game core, both on SURVEY.md §8(d) config 1 (one game, random
policy, game_tick only, random reset), measured in THIS container where the
reference is importable read-only.  bench.py divides the restatement's rate on
the GPU box's cores by this ratio to quote a reference-equivalent CPU rate.

    python3 -B tools/ref_ratio.py [--seconds 20] > profiles/ref_vs_pyoracle.json
"""
import argparse
import contextlib
import io
import json
import os
import platform
import random
import sys
import time

REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def reference_rate(seconds, seed=0, tick_limit=2000):
    sys.path.insert(0, REF)
    import numpy as np
    from SkillshotGame import SkillshotGame  # the reference game core (read-only import)
    rng = random.Random(seed)
    np.random.seed(seed)
    g = SkillshotGame(random_positions=True)
    steps = 0
    with contextlib.redirect_stdout(io.StringIO()):
        t0 = time.perf_counter()
        while True:
            for _ in range(1000):
                for pl in (g.player1, g.player2):  # do_actions order (SkillshotLearner.py:206-213)
                    pl.move_direction_float(rng.uniform(-1, 1))
                    pl.move_look_float(rng.uniform(-1, 1))
                    pl.move_shoot_projectile()
                g.game_tick()
                if not g.game_live or g.ticks >= tick_limit:
                    g.game_reset(random_positions=True)
            steps += 1000
            el = time.perf_counter() - t0
            if el >= seconds:
                return steps / el


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--seconds", type=float, default=20.0)
    a = p.parse_args()
    from oracle.cpu_bench import run_python
    ref, py = [], []
    for k in range(3):  # interleaved, median of three
        ref.append(reference_rate(a.seconds / 3, seed=k))
        py.append(run_python(a.seconds / 3, seed=k)["env_steps_per_s"])
    ref.sort()
    py.sort()
    print(json.dumps(dict(reference_env_steps_per_s=ref[1], pyoracle_env_steps_per_s=py[1],
                          ratio_pyoracle_over_reference=py[1] / ref[1], procedure="SURVEY.md 8(d) config 1, "
                          "1 process, game_tick + actions, median of 3", host=platform.processor() or "x86_64",
                          python=platform.python_version())))


if __name__ == "__main__":
    main()
