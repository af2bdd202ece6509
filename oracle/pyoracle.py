"""Pure-Python restatement of the Skillshot step (the second CPU restatement
SURVEY.md §4 asks for, beside oracle/skillshot_oracle.c).

TEST INFRASTRUCTURE ONLY: used by tests/ as an independent checker of the C
oracle and the golden fixtures, never by the product path.  Small batches only
(plain Python loops, one game at a time).

Restated from the normative semantics (SURVEY.md Appendix A / §8(a) rows
A3-A12) with CPython floats and `math`, so every fp64 operation is the one the
reference performs (same order, same libm calls, Python's round-half-even
`round`, floored `%`, `**` through libm pow):
  move_direction  Player.move_direction_float   Player.py:57-68  (+ :70-76)
  move_look       Player.move_look_float        Player.py:33-39
  shoot           Player.move_shoot_projectile  Player.py:78-89
  game_tick       SkillshotGame.game_tick       SkillshotGame.py:115-122,
                  Projectile.tick / move_forwards Projectile.py:38-53,
                  SkillshotGame.check_collision SkillshotGame.py:58-94
  features        SkillshotGame.get_state       SkillshotGame.py:124-166
  observe         SkillshotLearner.prepare_states :512-543 and the rewards
                  calculate_rewards_looking :575-588 / _simple :590-603
  step            do_actions (P1 then P2, :206-213) + game_tick + observe,
                  done = not live or ticks >= limit (:302)
State uses the engine's HBM layout when exchanged (load / arrays), so the
golden-replay harness (tests/golden_replay.py) drives it like the C oracle.
"""
import math

import numpy as np

BOARD = 250
PLAYER_SIDE, PROJ_SIDE = 5, 3
MOVE, LOOK, PROJ_SPEED, COOLDOWN = 3, 0.25, 5, 15
MAX_DIST = (2 * BOARD ** 2) ** 0.5  # SkillshotLearner.py:43


def _clamp_unit(v):
    # the reference's `1 if v >= 1 else v` then `-1 if v <= -1 else v`
    if v >= 1:
        return 1
    if v <= -1:
        return -1
    return v


def _fits(x, y, side):
    return 0 <= x and x + side <= BOARD and 0 <= y and y + side <= BOARD


def _gradient(r):
    return math.tan(-r + math.pi / 2)


def _line_point(g, lx, ly, cx, cy):
    return abs(g * cx - cy + (ly - g * lx)) / math.sqrt(g ** 2 + 1)


def _point_point(ax, ay, bx, by):
    return ((ax - bx) ** 2 + (ay - by) ** 2) ** 0.5


def _quirk_angle(r):
    # `(r % 2 * np.pi) / 2 * np.pi` evaluated left to right (SkillshotLearner.py:529)
    return ((r % 2) * math.pi) / 2 * math.pi


class Game:
    """One game's state as plain Python values (players indexed 0 / 1)."""
    __slots__ = ("x", "y", "rot", "qx", "qy", "qrot", "qcd", "qage", "qvalid", "ticks", "live", "winner")

    def __init__(self):
        self.x, self.y, self.rot = [50, 200], [50, 200], [0.0, 0.0]
        self.qx, self.qy, self.qrot = [0, 0], [0, 0], [0.0, 0.0]
        self.qcd, self.qage, self.qvalid = [0, 0], [0, 0], [False, False]
        self.ticks, self.live, self.winner = 0, True, 0

    # -- player actions
    def move_direction(self, p, speed):
        s = _clamp_unit(speed)
        sn, cs = math.sin(self.rot[p]), math.cos(self.rot[p])
        nx = int(round(self.x[p] - sn * MOVE * s))
        ny = int(round(self.y[p] - cs * MOVE * s))
        if _fits(nx, ny, PLAYER_SIDE):
            self.x[p], self.y[p] = nx, ny

    def move_look(self, p, angle):
        self.rot[p] += _clamp_unit(angle) * LOOK

    def shoot(self, p):
        if self.qcd[p] <= 0:
            self.qx[p], self.qy[p], self.qrot[p] = self.x[p], self.y[p], self.rot[p]
            self.qvalid[p], self.qcd[p], self.qage[p] = True, COOLDOWN, 0

    # -- game
    def _projectile_tick(self, p):
        nx = int(round(self.qx[p] - math.sin(self.qrot[p]) * PROJ_SPEED))
        ny = int(round(self.qy[p] - math.cos(self.qrot[p]) * PROJ_SPEED))
        if self.qvalid[p] and _fits(nx, ny, PROJ_SIDE):
            self.qx[p], self.qy[p] = nx, ny
        else:
            self.qvalid[p] = False
        self.qcd[p] -= 1
        self.qage[p] += 1

    def _hit(self, p):
        """player p touched by the opponent's projectile: some corner of the
        projectile box (x in {qx+3, qx}, y in {qy, qy-3}) inside p's box"""
        q = 1 - p
        if not self.qvalid[q]:
            return False
        xs = (self.qx[q] + PROJ_SIDE, self.qx[q])
        ys = (self.qy[q], self.qy[q] - PROJ_SIDE)
        return any(self.x[p] <= cx <= self.x[p] + PLAYER_SIDE and self.y[p] <= cy <= self.y[p] + PLAYER_SIDE
                   for cx in xs for cy in ys)

    def check_collision(self):
        for p in (0, 1):  # player 1 first; the first hit ends the game
            if self._hit(p):
                self.winner, self.live = p + 1, False
                return p + 1
        return 0

    def game_tick(self):
        if self.live:
            self.ticks += 1
            self._projectile_tick(0)
            self._projectile_tick(1)
            self.check_collision()

    # -- observation
    def _future(self, p):
        o = 1 - p
        if not self.qvalid[p]:
            return False
        g = _gradient(self.qrot[p])
        x_dir = 1 if -math.sin(self.qrot[p]) >= 0 else -1
        yi = self.qy[p] - g * self.qx[p]
        for xb in (self.qx[p], self.qx[p] + PROJ_SIDE):
            if (xb - self.qx[p]) * x_dir < 0:
                continue
            for X in (self.x[o], self.x[o] + PLAYER_SIDE):
                if self.y[o] <= g * X + yi <= self.y[o] + PLAYER_SIDE:
                    return True
        return False

    def features(self, p):
        """get_state's per-player values in the engine's FEATURE_KEYS order"""
        o = 1 - p
        gp, gq = _gradient(self.rot[p]), _gradient(self.qrot[p])
        return [gp, 1 if -math.sin(self.rot[p]) >= 0 else -1,
                _line_point(gp, self.x[p], self.y[p], self.x[o], self.y[o]),
                _point_point(self.x[p], self.y[p], self.x[o], self.y[o]),
                self.x[p], self.y[p], self.rot[p], self.qcd[p],
                gq, 1 if -math.sin(self.qrot[p]) >= 0 else -1,
                _line_point(gq, self.qx[p], self.qy[p], self.x[o], self.y[o]),
                self.qx[p], self.qy[p], self.qrot[p], self.qage[p], self.qvalid[p],
                _point_point(self.qx[p], self.qy[p], self.x[o], self.y[o]),
                self._future(p)]

    def observe(self, p, reward_kind=0):
        f = self.features(p)
        obs = [f[2] / MAX_DIST, f[3] / MAX_DIST, f[4] / BOARD, f[5] / BOARD, _quirk_angle(f[6]),
               f[7] / COOLDOWN, f[16] / MAX_DIST, f[11] / BOARD, f[12] / BOARD, _quirk_angle(f[13]),
               f[10] / MAX_DIST, int(f[17])]
        if reward_kind == 1:  # simple: own projectile distance minus the opponent's
            reward = f[16] - self.features(1 - p)[16]
        else:  # looking: -(own line distance) / board size
            reward = -f[2] / BOARD
        return obs, reward


class PyOracle:
    """N games with the engine-protocol methods of tests/golden_replay.replay."""

    def __init__(self, n):
        self.games = [Game() for _ in range(n)]

    def load(self, a):
        pos, rot, qpos, qrot = (np.asarray(a[k]) for k in ("pos", "rot", "qpos", "qrot"))
        qcdage, misc = np.asarray(a["qcdage"]), np.asarray(a["misc"])
        for i, g in enumerate(self.games):
            g.x = [int(pos[i, 0]), int(pos[i, 2])]
            g.y = [int(pos[i, 1]), int(pos[i, 3])]
            g.rot = [float(rot[i, 0]), float(rot[i, 1])]
            g.qx = [int(qpos[i, 0]), int(qpos[i, 2])]
            g.qy = [int(qpos[i, 1]), int(qpos[i, 3])]
            g.qrot = [float(qrot[i, 0]), float(qrot[i, 1])]
            g.qcd = [int(qcdage[i, 0]), int(qcdage[i, 2])]
            g.qage = [int(qcdage[i, 1]), int(qcdage[i, 3])]
            flags = int(misc[i, 1]) & 0xFFFFFFFF
            g.qvalid = [bool(flags & 0xFF), bool((flags >> 8) & 0xFF)]
            g.live, g.winner = bool((flags >> 16) & 0xFF), (flags >> 24) & 0xFF
            g.ticks = int(misc[i, 0])

    def arrays(self):
        n = len(self.games)
        out = dict(pos=np.zeros((n, 4), np.int32), rot=np.zeros((n, 2)), qpos=np.zeros((n, 4), np.int32),
                   qrot=np.zeros((n, 2)), qcdage=np.zeros((n, 4), np.int32), misc=np.zeros((n, 2), np.int32))
        for i, g in enumerate(self.games):
            out["pos"][i] = (g.x[0], g.y[0], g.x[1], g.y[1])
            out["rot"][i] = g.rot
            out["qpos"][i] = (g.qx[0], g.qy[0], g.qx[1], g.qy[1])
            out["qrot"][i] = g.qrot
            out["qcdage"][i] = (g.qcd[0], g.qage[0], g.qcd[1], g.qage[1])
            flags = int(g.qvalid[0]) | (int(g.qvalid[1]) << 8) | (int(g.live) << 16) | (g.winner << 24)
            out["misc"][i] = (g.ticks, np.uint32(flags).view(np.int32))
        return out

    def move_direction(self, pid, speeds):
        for g, s in zip(self.games, np.broadcast_to(speeds, (len(self.games),))):
            g.move_direction(pid - 1, float(s))

    def move_look(self, pid, angles):
        for g, s in zip(self.games, np.broadcast_to(angles, (len(self.games),))):
            g.move_look(pid - 1, float(s))

    def shoot(self, pid, mask=None):
        for i, g in enumerate(self.games):
            if mask is None or mask[i]:
                g.shoot(pid - 1)

    def game_tick(self):
        for g in self.games:
            g.game_tick()

    def observe(self, reward_kind=0):
        n = len(self.games)
        obs, rew = np.zeros((2, n, 12)), np.zeros((2, n))
        for i, g in enumerate(self.games):
            for p in (0, 1):
                obs[p, i], rew[p, i] = g.observe(p, reward_kind)
        return obs, rew

    def features(self):
        return np.array([[g.features(p) for p in (0, 1)] for g in self.games], dtype=np.float64)

    def step(self, actions, tick_limit=2000, reward_kind=0):
        """the learner protocol for one tick (no auto-reset); actions [2, N, 2]
        float32, promoted exactly to Python floats"""
        a = np.asarray(actions, dtype=np.float32)
        for i, g in enumerate(self.games):
            for p in (0, 1):
                g.move_direction(p, float(a[p, i, 0]))
                g.move_look(p, float(a[p, i, 1]))
                g.shoot(p)
            g.game_tick()
        obs, rew = self.observe(reward_kind)
        done = np.array([(not g.live) or g.ticks >= tick_limit for g in self.games], np.uint8)
        winner = np.array([g.winner for g in self.games], np.uint8)
        return dict(obs=obs, reward=rew, done=done, winner=winner)
