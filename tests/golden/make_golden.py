"""Generate golden trajectory fixtures by running the REFERENCE game core.

Test infrastructure only.  Run in the build container (where the read-only
reference checkout lives at /root/reference):

    python3 -B tests/golden/make_golden.py

It imports the reference's game core (SkillshotGame.py / Player.py /
Projectile.py) and, because SkillshotLearner.py imports TensorFlow at module
scope (SkillshotLearner.py:5) which is not installed, it AST-extracts only the
TF-free learner methods needed for the observation and reward
(prepare_states SkillshotLearner.py:512-543, calculate_rewards_looking :575-588,
calculate_rewards_simple :590-603) and binds them to a stub object.  Nothing
from the reference is written to the repo: only the resulting numbers (.npz).

Drive conventions (SURVEY.md §7 hard part 2): actions are float32 values
promoted exactly to Python floats, so the reference runs in pure fp64.  Per
tick the learner protocol is applied (SkillshotLearner.do_actions :206-213 for
player 1 then player 2, then game_tick, then get_state), except for the
"raw" scenarios which call the Player methods individually with a shoot mask
(the keyboard/playable protocol, skillshot_playable.py:51-64).
"""
import ast
import contextlib
import io
import math
import os
import random
import sys

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)

import SkillshotGame as _sg  # noqa: E402  (reference game core)

SkillshotGame = _sg.SkillshotGame


def _load_learner_methods():
    src = open(os.path.join(REF, "SkillshotLearner.py")).read()
    tree = ast.parse(src)
    wanted = {"prepare_states", "calculate_rewards_looking", "calculate_rewards_simple", "calculate_rewards",
              "do_actions"}
    fns = []
    for node in tree.body:
        if isinstance(node, ast.ClassDef) and node.name == "SkillshotLearner":
            for item in node.body:
                if isinstance(item, ast.FunctionDef) and item.name in wanted:
                    item.decorator_list = []
                    fns.append(item)
    mod = ast.Module(body=fns, type_ignores=[])
    ns = {"np": np}
    exec(compile(mod, "SkillshotLearner.py(extract)", "exec"), ns)
    return {k: ns[k] for k in wanted}


_M = _load_learner_methods()


class LearnerStub:
    """Exposes exactly the attributes the extracted methods read
    (SkillshotLearner.py:41-43)."""

    def __init__(self, game):
        self.game_environment = game
        self.player_ids = (1, 2)
        self.max_dist_normaliser = (2 * (250 ** 2)) ** 0.5

    def prepare_states(self, states, pid):
        return _M["prepare_states"](self, states, pid)

    def rewards_looking(self, states):
        with contextlib.redirect_stdout(io.StringIO()):
            return _M["calculate_rewards_looking"](self, states)

    def rewards_simple(self, states):
        return _M["calculate_rewards_simple"](self, states)

    def rewards_full(self, states):
        """calculate_rewards (:605-661) over an episode's post-tick states."""
        try:
            r = _M["calculate_rewards"](self, states)
        except IndexError:
            return None, np.array([[st[1]["projectile_dist_opponent"], st[2]["projectile_dist_opponent"]]
                                   for st in states], dtype=np.float64)  # the reference raised
        return (np.array([[x[1], x[2]] for x in r], dtype=np.float64),
                np.array([[st[1]["projectile_dist_opponent"], st[2]["projectile_dist_opponent"]]
                          for st in states], dtype=np.float64))

    def do_actions(self, pid, pred):
        return _M["do_actions"](self, pid, pred)


def snapshot(g):
    p = (g.player1, g.player2)
    return dict(
        pos=[[int(pl.pos[0]), int(pl.pos[1])] for pl in p],
        rot=[float(pl.rotation) for pl in p],
        qpos=[[int(pl.projectile.pos[0]), int(pl.projectile.pos[1])] for pl in p],
        qrot=[float(pl.projectile.rotation) for pl in p],
        qcd=[int(pl.projectile.cooldown_current) for pl in p],
        qage=[int(pl.projectile.age) for pl in p],
        qvalid=[int(bool(pl.projectile.valid)) for pl in p],
        ticks=int(g.ticks), live=int(bool(g.game_live)), winner=int(g.winner_id))


def features(learner, g):
    st = g.get_state()
    obs = [learner.prepare_states([st], pid)[0] for pid in (1, 2)]
    rl = learner.rewards_looking([st])[0]
    rs = learner.rewards_simple([st])[0]
    return (np.array(obs, dtype=np.float64),
            np.array([rl[1], rl[2]], dtype=np.float64),
            np.array([rs[1], rs[2]], dtype=np.float64))


def set_state(g, init):
    """Write an explicit state into a reference game object (plain attributes)."""
    for i, pl in enumerate((g.player1, g.player2)):
        pl.pos = [int(init["pos"][i][0]), int(init["pos"][i][1])]
        pl.rotation = init["rot"][i]
        q = pl.projectile
        q.pos = [int(init["qpos"][i][0]), int(init["qpos"][i][1])]
        q.rotation = init["qrot"][i]
        q.cooldown_current = int(init["qcd"][i])
        q.age = int(init["qage"][i])
        q.valid = bool(init["qvalid"][i])
    g.ticks = int(init.get("ticks", 0))
    g.game_live = bool(init.get("live", 1))
    g.winner_id = int(init.get("winner", 0))


def run_env(game, actions, tick_limit, protocol="learner", shoot=None, run_after_done=0):
    """Roll one reference env.  actions: f32 [T,2,2].  Returns per-tick records.

    learner protocol stops once done (SkillshotLearner.py:302); with
    run_after_done>0 the raw protocol keeps stepping after the game ended to
    pin that dead games do not tick (SkillshotGame.py:117) while moves apply.
    """
    learner = LearnerStub(game)
    snaps = [snapshot(game)]
    states = []
    o, rl, rs = features(learner, game)
    obs, rew, rsim = [o], [rl], [rs]
    done_at = None
    T = actions.shape[0]
    t = 0
    with contextlib.redirect_stdout(io.StringIO()):
        while t < T:
            if protocol == "learner":
                if not (game.game_live and game.ticks < tick_limit):
                    break
                for pid in (1, 2):
                    a = actions[t, pid - 1]
                    learner.do_actions(pid, [float(a[0]), float(a[1])])
            else:
                if done_at is not None and t >= done_at + run_after_done:
                    break
                for pid in (1, 2):
                    pl = game.get_player_by_id(pid)
                    a = actions[t, pid - 1]
                    pl.move_direction_float(float(a[0]))
                    pl.move_look_float(float(a[1]))
                    if shoot[t, pid - 1]:
                        pl.move_shoot_projectile()
            game.game_tick()
            t += 1
            states.append(game.get_state())
            snaps.append(snapshot(game))
            o, rl, rs = features(learner, game)
            obs.append(o)
            rew.append(rl)
            rsim.append(rs)
            if done_at is None and not (game.game_live and game.ticks < tick_limit):
                done_at = t
    full = learner.rewards_full(states) if protocol == "learner" and states else (None, None)
    return snaps, obs, rew, rsim, t, full


def pack(name, inits, acts, results, tick_limit, protocol, shoot=None, note=""):
    E = len(results)
    Tm = max(r[4] for r in results)
    if protocol == "learner":
        # calculate_rewards (:605-661) over states[1:] of each episode; NaN rows
        # pad, and an episode on which the reference raises is all-NaN
        rf = np.full((E, max(Tm, 1), 2), np.nan)
        rd = np.full((E, max(Tm, 1), 2), np.nan)
        for e, r in enumerate(results):
            if r[5][0] is not None:
                rf[e, :r[5][0].shape[0]] = r[5][0]
            if r[5][1] is not None:
                rd[e, :r[5][1].shape[0]] = r[5][1]
        out_full = (rf, rd)
    else:
        out_full = None
    out = dict(
        scenario=np.array(name), protocol=np.array(protocol), note=np.array(note),
        tick_limit=np.int32(tick_limit), numpy_version=np.array(np.__version__),
        n_steps=np.array([r[4] for r in results], dtype=np.int32),
        actions=np.stack([a[:max(Tm, 1)] for a in acts]).astype(np.float32),
    )
    if shoot is not None:
        out["shoot"] = np.stack([s[:max(Tm, 1)] for s in shoot]).astype(np.uint8)

    def field(key, dtype):
        arr = []
        for snaps, *_ in results:
            seq = [s[key] for s in snaps]
            seq += [seq[-1]] * (Tm + 1 - len(seq))
            arr.append(seq)
        return np.array(arr, dtype=dtype)

    out["pos"] = field("pos", np.int32)
    out["rot"] = field("rot", np.float64)
    out["qpos"] = field("qpos", np.int32)
    out["qrot"] = field("qrot", np.float64)
    out["qcd"] = field("qcd", np.int32)
    out["qage"] = field("qage", np.int32)
    out["qvalid"] = field("qvalid", np.uint8)
    out["ticks"] = field("ticks", np.int32)
    out["live"] = field("live", np.uint8)
    out["winner"] = field("winner", np.uint8)

    def series(idx):
        arr = []
        for r in results:
            seq = list(r[idx])
            seq += [seq[-1]] * (Tm + 1 - len(seq))
            arr.append(np.stack(seq))
        return np.stack(arr)

    if out_full is not None:
        # the reference's projectile_dist_opponent per post-tick state: its
        # value depends on the coordinates' Python types (int ** 0.5 is libm
        # pow, np.int64 ** 0.5 is numpy's sqrt), so the reward is pinned on it
        out["reward_full"], out["reward_full_dist"] = out_full
    out["obs"] = series(1)
    out["reward"] = series(2)
    out["reward_simple"] = series(3)
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **out)
    print(f"{name}: E={E} max_ticks={Tm} -> {os.path.getsize(path)} bytes")


def f32_uniform(rng, shape, lo=-1.0, hi=1.0):
    return np.array([rng.uniform(lo, hi) for _ in range(int(np.prod(shape)))],
                    dtype=np.float32).reshape(shape)


def fixed_init():
    return dict(pos=[[50, 50], [200, 200]], rot=[0, 0], qpos=[[0, 0], [0, 0]], qrot=[0, 0],
                qcd=[0, 0], qage=[0, 0], qvalid=[0, 0])


def scenario_random_policy(name, E, T, tick_limit, start, seed):
    rng = random.Random(seed)
    inits, acts, results = [], [], []
    for e in range(E):
        if start == "fixed":
            g = SkillshotGame()
        elif start == "numpy":
            # the reference's own random start (np.int64 positions, SkillshotGame.py:15)
            np.random.seed(seed * 1000 + e)
            g = SkillshotGame(random_positions=True)
        else:
            g = SkillshotGame()
            init = fixed_init()
            init["pos"] = [[rng.randrange(25, 225), rng.randrange(25, 225)] for _ in range(2)]
            set_state(g, init)
        a = f32_uniform(rng, (T, 2, 2))
        inits.append(snapshot(g))
        acts.append(a)
        results.append(run_env(g, a, tick_limit))
    pack(name, inits, acts, results, tick_limit, "learner",
         note=f"random policy, {start} start, seed {seed}")


def scenario_ties():
    # rotation 0 => sin=0, cos=1; a0=+-0.5 => y -+ 1.5 exactly: half-even ties
    # (y=50 -> 48.5 -> 48 ; y=51 -> 49.5 -> 50).
    inits, acts, results = [], [], []
    T = 40
    for e, (y0, s) in enumerate([(50, 0.5), (51, 0.5), (52, -0.5), (53, -0.5), (100, 0.5), (101, -0.5)]):
        g = SkillshotGame()
        init = fixed_init()
        init["pos"] = [[60 + e, y0], [180, 200 - e]]
        set_state(g, init)
        a = np.zeros((T, 2, 2), dtype=np.float32)
        a[:, 0, 0] = s
        a[:, 1, 0] = -s
        a[::7, 0, 1] = 0.0
        inits.append(snapshot(g))
        acts.append(a)
        results.append(run_env(g, a, 2000))
    pack("ties", inits, acts, results, 2000, "learner", note="exact .5 rounding ties at rotation 0")


def scenario_walls(seed=7):
    rng = random.Random(seed)
    inits, acts, results = [], [], []
    T = 200
    corners = [[0, 0], [245, 0], [0, 245], [245, 245], [2, 120], [243, 120], [120, 1], [120, 244]]
    for e, c in enumerate(corners):
        g = SkillshotGame()
        init = fixed_init()
        init["pos"] = [c, [125, 125]]
        init["rot"] = [rng.uniform(-4, 4), rng.uniform(-4, 4)]
        set_state(g, init)
        a = f32_uniform(rng, (T, 2, 2))
        a[:, 0, 0] = np.where(a[:, 0, 0] > -0.5, 1.0, a[:, 0, 0])  # push into the wall mostly
        a[:, 0, 1] = a[:, 0, 1] * 0.1
        inits.append(snapshot(g))
        acts.append(a)
        results.append(run_env(g, a, 2000))
    pack("walls", inits, acts, results, 2000, "learner", note="wall clamping and projectile invalidation")


def scenario_negrot(seed=11):
    rng = random.Random(seed)
    inits, acts, results = [], [], []
    T = 300
    for e in range(6):
        g = SkillshotGame()
        init = fixed_init()
        init["pos"] = [[rng.randrange(25, 225), rng.randrange(25, 225)] for _ in range(2)]
        set_state(g, init)
        a = f32_uniform(rng, (T, 2, 2))
        a[:, :, 1] = f32_uniform(rng, (T, 2), -1.0, -0.2)
        inits.append(snapshot(g))
        acts.append(a)
        results.append(run_env(g, a, 2000))
    pack("negrot", inits, acts, results, 2000, "learner", note="negative rotations (floored %)")


def scenario_bigrot(seed=29):
    """Rotations far from the game's usual +-500 (settable through the class
    API's Player.rotation): 1e3 .. 1e8 rad, on both sides of the fast sin/cos
    path's reduction range (|r| < 2^20 pi/2 = 1,647,099.3), with the
    projectiles inheriting them when fired."""
    rng = random.Random(seed)
    inits, acts, results = [], [], []
    T = 200
    mags = [1.0e3, 7.5e4, 1.6e6, 1647099.0, 1647100.0, 3.3e6, 2.0e7, 1.0e8]
    for e, mag in enumerate(mags):
        g = SkillshotGame()
        init = fixed_init()
        init["pos"] = [[rng.randrange(25, 225), rng.randrange(25, 225)] for _ in range(2)]
        init["rot"] = [mag * (1 if e % 2 else -1) + rng.uniform(-1, 1), -mag + rng.uniform(-1, 1)]
        set_state(g, init)
        a = f32_uniform(rng, (T, 2, 2))
        inits.append(snapshot(g))
        acts.append(a)
        results.append(run_env(g, a, 2000))
    pack("bigrot", inits, acts, results, 2000, "learner", note="rotations of 1e3 .. 1e8 rad (class-API settable)")


def scenario_offboard(seed=31):
    """Players and projectiles placed outside the 250 x 250 board (the class
    API sets positions freely; Player.check_pos_valid only refuses moves):
    negative and > 250 coordinates, a live projectile off the board, some
    games starting with a projectile already in flight toward the other
    player."""
    rng = random.Random(seed)
    inits, acts, results = [], [], []
    T = 150
    places = [([-40, 100], [120, 120]), ([300, -20], [10, 240]), ([125, 260], [125, -30]),
              ([-5, -5], [255, 255]), ([0, 245], [245, 0]), ([-100, 400], [60, 60])]
    for e, (p1, p2) in enumerate(places):
        g = SkillshotGame()
        init = fixed_init()
        init["pos"] = [p1, p2]
        init["rot"] = [rng.uniform(-4, 4), rng.uniform(-4, 4)]
        if e % 2 == 0:  # player 1's projectile in flight, possibly off the board
            init["qpos"] = [[p1[0] + rng.randrange(-30, 30), p1[1] + rng.randrange(-30, 30)], [0, 0]]
            init["qrot"] = [rng.uniform(-4, 4), 0.0]
            init["qcd"] = [rng.randrange(-5, 15), 0]
            init["qage"] = [rng.randrange(0, 20), 0]
            init["qvalid"] = [1, 0]
        set_state(g, init)
        a = f32_uniform(rng, (T, 2, 2))
        inits.append(snapshot(g))
        acts.append(a)
        results.append(run_env(g, a, 2000))
    pack("offboard", inits, acts, results, 2000, "learner", note="positions / projectiles outside the board")


def scenario_clamp(seed=13):
    rng = random.Random(seed)
    inits, acts, results = [], [], []
    T = 150
    specials = np.array([1.0, -1.0, 1.5, -1.5, 3e38, -3e38, np.inf, -np.inf, 0.9999999, -0.9999999,
                         0.0, -0.0, 1.0000001, 2.0, -7.25], dtype=np.float32)
    for e in range(6):
        g = SkillshotGame()
        init = fixed_init()
        init["pos"] = [[rng.randrange(25, 225), rng.randrange(25, 225)] for _ in range(2)]
        set_state(g, init)
        a = f32_uniform(rng, (T, 2, 2), -3.0, 3.0)
        mask = np.array([rng.random() < 0.4 for _ in range(T * 4)]).reshape(T, 2, 2)
        picks = np.array([specials[rng.randrange(len(specials))] for _ in range(T * 4)],
                         dtype=np.float32).reshape(T, 2, 2)
        a = np.where(mask, picks, a).astype(np.float32)
        inits.append(snapshot(g))
        acts.append(a)
        results.append(run_env(g, a, 2000))
    pack("clamp", inits, acts, results, 2000, "learner", note="action clamping incl. +-1, +-inf, out of range")


def _both_hit(g):
    hits = []
    for pl, q in ((g.player1, g.player2.projectile), (g.player2, g.player1.projectile)):
        h = False
        if q.valid:
            L, R, Tp, B = pl.pos[0], pl.pos[0] + 5, pl.pos[1], pl.pos[1] + 5
            for X in (q.pos[0] + 3, q.pos[0]):
                for Y in (q.pos[1], q.pos[1] - 3):
                    if L <= X <= R and Tp <= Y <= B:
                        h = True
        hits.append(h)
    return hits


def scenario_both_hit(seed=17, want=6):
    """Search for trajectories in which BOTH players are hit on the same tick
    (check_collision's P1 precedence, SkillshotGame.py:60-94)."""
    rng = random.Random(seed)
    inits, acts, results = [], [], []
    tries = 0
    while len(results) < want and tries < 200000:
        tries += 1
        g = SkillshotGame()
        init = fixed_init()
        x1, y1 = rng.randrange(60, 180), rng.randrange(60, 180)
        dx, dy = rng.randrange(-25, 26), rng.randrange(-25, 26)
        init["pos"] = [[x1, y1], [x1 + dx, y1 + dy]]
        ang = math.atan2(-dx, -dy)  # facing the opponent: dir = (-sin r, -cos r)
        init["rot"] = [ang + rng.uniform(-0.05, 0.05), ang + math.pi + rng.uniform(-0.05, 0.05)]
        set_state(g, init)
        T = 30
        a = np.zeros((T, 2, 2), dtype=np.float32)
        a[:, :, :] = f32_uniform(rng, (T, 2, 2), -0.05, 0.05)
        # dry run on a copy
        g2 = SkillshotGame()
        set_state(g2, init)
        ok = False
        with contextlib.redirect_stdout(io.StringIO()):
            for t in range(T):
                for pid in (1, 2):
                    pl = g2.get_player_by_id(pid)
                    pl.move_direction_float(float(a[t, pid - 1, 0]))
                    pl.move_look_float(float(a[t, pid - 1, 1]))
                    pl.move_shoot_projectile()
                for pl in (g2.player1, g2.player2):
                    pl.projectile.tick()
                hb = _both_hit(g2)
                if hb[0] or hb[1]:
                    ok = hb[0] and hb[1]
                    break
        if not ok:
            continue
        inits.append(snapshot(g))
        acts.append(a)
        results.append(run_env(g, a, 2000))
    assert len(results) == want, f"found only {len(results)} both-hit cases"
    pack("both_hit", inits, acts, results, 2000, "learner", note=f"simultaneous hits, found in {tries} tries")


def scenario_raw(seed=19):
    """Per-method protocol with a shoot mask: cooldown goes negative, and the
    env keeps being driven after the game ended (dead games do not tick)."""
    rng = random.Random(seed)
    inits, acts, shoots, results = [], [], [], []
    T = 900
    for e in range(6):
        g = SkillshotGame()
        init = fixed_init()
        init["pos"] = [[rng.randrange(25, 225), rng.randrange(25, 225)] for _ in range(2)]
        if e == 0:
            init["pos"] = [[100, 100], [100, 120]]
        set_state(g, init)
        a = f32_uniform(rng, (T, 2, 2))
        p_shoot = [0.02, 0.3, 0.0, 0.05, 1.0, 0.1][e]
        s = np.array([rng.random() < p_shoot for _ in range(T * 2)], dtype=np.uint8).reshape(T, 2)
        inits.append(snapshot(g))
        acts.append(a)
        shoots.append(s)
        results.append(run_env(g, a, 2 ** 31 - 1, protocol="raw", shoot=s, run_after_done=40))
    pack("raw", inits, acts, results, 2 ** 31 - 1, "raw", shoot=shoots,
         note="per-method calls, sparse shooting, stepping continues 40 ticks after game end")


if __name__ == "__main__" and "--only" in sys.argv:  # one scenario: --only NAME (e.g. bigrot)
    globals()["scenario_" + sys.argv[sys.argv.index("--only") + 1]]()
elif __name__ == "__main__" and "--boards" not in sys.argv:
    scenario_random_policy("fixed_random", 8, 2000, 2000, "fixed", 1)
    scenario_random_policy("numpy_start", 8, 2000, 2000, "numpy", 2)
    scenario_random_policy("int_start_limit200", 12, 200, 200, "int", 3)
    scenario_ties()
    scenario_walls()
    scenario_negrot()
    scenario_clamp()
    scenario_both_hit()
    scenario_raw()


def scenario_boards():
    """get_board (SkillshotGame.py:36-56) and raw get_state dicts (:136-166) on
    states sampled from reference trajectories (F4 row / class-API parity)."""
    rng = random.Random(23)
    states, boards, feats, general = [], [], [], []
    keys = ["player_grad", "player_x_dir", "player_path_dist_opponent", "player_dist_opponent",
            "player_pos_x", "player_pos_y", "player_rotation", "projectile_cooldown", "projectile_grad",
            "projectile_x_dir", "projectile_path_dist_opponent", "projectile_pos_x", "projectile_pos_y",
            "projectile_rotation", "projectile_age", "projectile_valid", "projectile_dist_opponent",
            "projectile_future_collision_opponent"]
    with contextlib.redirect_stdout(io.StringIO()):
        for e in range(6):
            g = SkillshotGame()
            init = fixed_init()
            init["pos"] = [[rng.randrange(0, 246), rng.randrange(0, 246)] for _ in range(2)]
            set_state(g, init)
            learner = LearnerStub(g)
            for t in range(120):
                for pid in (1, 2):
                    learner.do_actions(pid, [rng.uniform(-1, 1), rng.uniform(-1, 1)])
                g.game_tick()
                if t % 20 == 7:
                    snap = snapshot(g)
                    st = g.get_state()
                    states.append(snap)
                    boards.append(g.get_board().astype(np.int8))
                    feats.append([[float(st[pid][k]) for k in keys] for pid in (1, 2)])
                    general.append([int(bool(st["game_live"])), int(st["ticks"]), int(st["game_winner"])])
    out = dict(
        pos=np.array([s["pos"] for s in states], np.int32), rot=np.array([s["rot"] for s in states]),
        qpos=np.array([s["qpos"] for s in states], np.int32), qrot=np.array([s["qrot"] for s in states]),
        qcd=np.array([s["qcd"] for s in states], np.int32), qage=np.array([s["qage"] for s in states], np.int32),
        qvalid=np.array([s["qvalid"] for s in states], np.uint8),
        ticks=np.array([s["ticks"] for s in states], np.int32), live=np.array([s["live"] for s in states], np.uint8),
        winner=np.array([s["winner"] for s in states], np.uint8),
        board=np.stack(boards), features=np.array(feats, np.float64), general=np.array(general, np.int64),
        numpy_version=np.array(np.__version__))
    path = os.path.join(OUT, "boards.npz")
    np.savez_compressed(path, **out)
    print(f"boards: {len(states)} states -> {os.path.getsize(path)} bytes")


if __name__ == "__main__" and "--only" not in sys.argv:
    scenario_boards()
