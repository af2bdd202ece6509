"""The reference's own per-call protocol through the class-API shim on
libskillshot's CPU backend: SURVEY.md §8(d) config 1 (one game, random policy
random.Random(seed).uniform(-1, 1) in do_actions order, game_tick, random
reset on done or at 2,000 ticks, hit prints silenced), tick only and with
get_state() per tick (the obs source, SkillshotGame.py:136-166) — the two
rows of BASELINE.md (59.2k / 18.9k env-steps/s per core for the reference in
the survey container).

    python3 -B tools/class_api_bench.py [--seconds 6] [--reference]

--reference also times the reference game core (imported read-only from
/root/reference; only where it exists, i.e. never on the GPU box) with the
same procedure, interleaved, so the ratio is same-host."""
import argparse
import contextlib
import io
import json
import os
import platform
import random
import sys
import time

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rate(make_game, seconds, seed, with_state, tick_limit=2000):
    import numpy as np
    rng = random.Random(seed)
    np.random.seed(seed)
    g = make_game()
    g.game_reset(random_positions=True)
    steps = 0
    with contextlib.redirect_stdout(io.StringIO()):
        t0 = time.perf_counter()
        while True:
            for _ in range(500):
                for pl in (g.player1, g.player2):  # do_actions order (SkillshotLearner.py:206-213)
                    pl.move_direction_float(rng.uniform(-1, 1))
                    pl.move_look_float(rng.uniform(-1, 1))
                    pl.move_shoot_projectile()
                g.game_tick()
                if with_state:
                    g.get_state()
                if not g.game_live or g.ticks >= tick_limit:
                    g.game_reset(random_positions=True)
            steps += 500
            el = time.perf_counter() - t0
            if el >= seconds:
                return steps / el


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--seconds", type=float, default=6.0)
    p.add_argument("--reference", action="store_true")
    a = p.parse_args()
    from skillshot_learning_amd import game
    makers = {"shim_cpu_backend": lambda: game.SkillshotGame(device="cpu")}
    if a.reference and os.path.isdir("/root/reference"):
        sys.path.insert(0, "/root/reference")
        from SkillshotGame import SkillshotGame as RefGame  # read-only import of the reference game core
        makers["reference"] = lambda: RefGame()
    out = {}
    for with_state in (False, True):
        key = "tick_and_get_state" if with_state else "tick_only"
        res = {k: [] for k in makers}
        for s in range(3):  # interleaved, median of three
            for k, mk in makers.items():
                res[k].append(rate(mk, a.seconds / 3, s, with_state))
        out[key] = {k: sorted(v)[1] for k, v in res.items()}
        if "reference" in out[key]:
            out[key]["ratio_shim_over_reference"] = out[key]["shim_cpu_backend"] / out[key]["reference"]
    out.update(procedure="SURVEY.md 8(d) config 1: one game, 1 process, random policy in do_actions order, "
                         "game_tick (+ get_state), random reset; median of 3 interleaved runs",
               backend="skillshot_learning_amd.game.SkillshotGame(device='cpu') -> libskillshot CPU backend",
               host=platform.processor() or "x86_64", python=platform.python_version(),
               reference_baseline_md={"tick_only": 59200, "tick_and_get_state": 18900})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
