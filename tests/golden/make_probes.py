"""Generate collision / future-collision probe fixtures from the REFERENCE.

Test infrastructure only.  Run in the build container (where the read-only
reference checkout lives at /root/reference):

    python3 -B tests/golden/make_probes.py

Each probe is a board written straight into a reference SkillshotGame
(make_golden.set_state) with the projectile placed within a few pixels of the
opponent box, so the inclusive corner tests of check_collision
(SkillshotGame.py:58-94) and the fp64 interval test of check_future_collision
(SkillshotGame.py:96-113) are exercised on and around their boundaries.
Rotations mix uniform draws, exact multiples of pi/4 (gradients 0, +-1 and
tan(pi/2) ~ 1.6e16) and "aimed" angles whose projectile line passes through an
opponent corner (the y comparison lands on the boundary up to fp64 rounding).

Recorded per probe: the reference's check_collision outcome (winner_id after
a call on a live game, 0 = no hit) and check_future_collision for both
projectiles; beside them the correctly rounded gradient tan(-qrot + pi/2)
(tests/cr_tan.py, 70-digit Decimal) and the future-collision decision under
it (`future_cr`): glibc's math.tan is not correctly rounded for ~0.3 % of
arguments, and the HIP kernels are pinned to the correctly rounded tan
(csrc/sk_tan_cr.hpp).  Only numbers are written (probes.npz).
"""
import contextlib
import io
import math
import os
import random
import sys

import numpy as np

sys.dont_write_bytecode = True
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as mg  # noqa: E402  (imports the reference game core)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cr_tan import cr_tan  # noqa: E402

N_PROBES = 6000


def _rotation(rng, qx, qy, ox, oy):
    kind = rng.random()
    if kind < 0.35:
        return rng.uniform(-4 * math.pi, 4 * math.pi)
    if kind < 0.55:
        return rng.randrange(-16, 17) * (math.pi / 4)
    # aim the projectile line at an opponent corner (Projectile.py:38-47: the
    # projectile moves by (-sin r, -cos r), so the direction to (dx, dy) is
    # r = atan2(-dx, -dy)); corners on both x bounds and both y bounds
    cx = ox + rng.choice((0, 5))
    cy = oy + rng.choice((0, 5))
    dx, dy = cx - qx, cy - qy
    if dx == 0 and dy == 0:
        return rng.uniform(-math.pi, math.pi)
    r = math.atan2(-dx, -dy)
    if rng.random() < 0.3:
        r += rng.choice((-1, 1)) * rng.choice((1e-15, 1e-12, 1e-9, 1e-6))
    return r + 2 * math.pi * rng.randrange(-2, 3)


def _future(g, q, o):
    """check_future_collision's compare (SkillshotGame.py:103-112) for a given gradient."""
    yi = float(q[1]) - g * float(q[0])
    return any(float(o[1]) <= g * float(X) + yi <= float(o[1] + 5) for X in (o[0], o[0] + 5))


def main():
    rng = random.Random(29)
    init_keys = ("pos", "rot", "qpos", "qrot", "qcd", "qage", "qvalid")
    rows = {k: [] for k in init_keys}
    hit, future, grad_cr, future_cr, glibc_is_cr = [], [], [], [], []
    with contextlib.redirect_stdout(io.StringIO()):
        for _ in range(N_PROBES):
            pos = [[rng.randrange(0, 246), rng.randrange(0, 246)] for _ in range(2)]
            qpos, qrot = [], []
            for p in range(2):
                o = pos[1 - p]
                near = rng.random() < 0.8
                span = 9 if near else 120
                qx = min(247, max(0, o[0] + rng.randrange(-span, span + 1)))
                qy = min(247, max(0, o[1] + rng.randrange(-span, span + 1)))
                qpos.append([qx, qy])
                qrot.append(_rotation(rng, qx, qy, o[0], o[1]))
            init = dict(pos=pos, rot=[rng.uniform(-math.pi, math.pi) for _ in range(2)], qpos=qpos, qrot=qrot,
                        qcd=[rng.randrange(-5, 16) for _ in range(2)], qage=[rng.randrange(0, 60) for _ in range(2)],
                        qvalid=[int(rng.random() < 0.85) for _ in range(2)])
            g = mg.SkillshotGame()
            mg.set_state(g, init)
            fut = [bool(g.check_future_collision(g.player1.projectile, g.player2)),
                   bool(g.check_future_collision(g.player2.projectile, g.player1))]
            g.game_live, g.winner_id = True, 0
            g.check_collision()
            hit.append(0 if g.game_live else int(g.winner_id))
            future.append(fut)
            gcr, fcr, gok = [], [], []
            for p in range(2):
                x = -qrot[p] + math.pi / 2
                gc = cr_tan(x)
                gcr.append(gc)
                gok.append(int(math.tan(x) == gc))
                fcr.append(int(bool(init["qvalid"][p]) and _future(gc, qpos[p], pos[1 - p])))
            grad_cr.append(gcr)
            future_cr.append(fcr)
            glibc_is_cr.append(gok)
            for k in init_keys:
                rows[k].append(init[k])
    out = dict(pos=np.array(rows["pos"], np.int32), rot=np.array(rows["rot"], np.float64),
               qpos=np.array(rows["qpos"], np.int32), qrot=np.array(rows["qrot"], np.float64),
               qcd=np.array(rows["qcd"], np.int32), qage=np.array(rows["qage"], np.int32),
               qvalid=np.array(rows["qvalid"], np.uint8), hit=np.array(hit, np.uint8),
               future=np.array(future, np.uint8), grad_cr=np.array(grad_cr, np.float64),
               future_cr=np.array(future_cr, np.uint8), glibc_is_cr=np.array(glibc_is_cr, np.uint8))
    path = os.path.join(mg.OUT, "probes.npz")
    np.savez_compressed(path, **out)
    h = out["hit"]
    print(f"probes: {N_PROBES} boards, hits p1={int((h == 1).sum())} p2={int((h == 2).sum())}, "
          f"future={int(out['future'].sum())}, glibc tan not CR on {int((out['glibc_is_cr'] == 0).sum())}, "
          f"flags differing under CR tan {int((out['future'] != out['future_cr']).sum())} "
          f"-> {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
