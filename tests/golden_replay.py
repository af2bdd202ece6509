"""Replay the reference golden fixtures (tests/golden/*.npz) through any
batched engine exposing the per-method / fused-step API, and compare.

Used by the oracle pin (CPU) and by the GPU parity tests, so the oracle and the
HIP path are held to the same fixtures.
"""
import glob
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fixture_names():
    """Trajectory fixtures (boards.npz and probes.npz hold single states, see
    test_board_cpu / test_closed_forms_cpu)."""
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz"))
                  if os.path.basename(p) not in SINGLE_STATE)


SINGLE_STATE = ("boards.npz", "probes.npz")


def probe_state(d):
    """Engine-layout arrays of the probe boards (probes.npz): live game, tick 0, no winner."""
    n = d["pos"].shape[0]
    zero = np.zeros(n, np.uint8)
    return dict(pos=d["pos"].reshape(n, 4), rot=d["rot"], qpos=d["qpos"].reshape(n, 4), qrot=d["qrot"],
                qcdage=np.stack([d["qcd"][:, 0], d["qage"][:, 0], d["qcd"][:, 1], d["qage"][:, 1]], -1),
                misc=np.stack([np.zeros(n, np.int32), _flags(d["qvalid"], zero + 1, zero)], -1))


def load(name):
    d = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
    return {k: d[k] for k in d.files}


def _flags(qvalid, live, winner):
    qv = qvalid.astype(np.uint32)
    f = (qv[..., 0] & 0xFF) | ((qv[..., 1] & 0xFF) << 8) | ((live.astype(np.uint32) & 0xFF) << 16) | \
        ((winner.astype(np.uint32) & 0xFF) << 24)
    return f.astype(np.uint32).view(np.int32)


def state_at(d, t):
    """Engine-layout state arrays of all envs at tick index t."""
    E = d["pos"].shape[0]
    return dict(
        pos=d["pos"][:, t].reshape(E, 4).astype(np.int32),
        rot=d["rot"][:, t].reshape(E, 2).astype(np.float64),
        qpos=d["qpos"][:, t].reshape(E, 4).astype(np.int32),
        qrot=d["qrot"][:, t].reshape(E, 2).astype(np.float64),
        qcdage=np.stack([d["qcd"][:, t, 0], d["qage"][:, t, 0], d["qcd"][:, t, 1], d["qage"][:, t, 1]],
                        -1).astype(np.int32),
        misc=np.stack([d["ticks"][:, t], _flags(d["qvalid"][:, t], d["live"][:, t], d["winner"][:, t])],
                      -1).astype(np.int32),
    )


OBS_TOL = 1e-5  # SURVEY.md §8(a) parity target for obs/reward, relative to max(1,|ref|)


def compare_state(got, want, active, where):
    """Bit-exact comparison of every state field for envs with active=True."""
    for k in ("pos", "rot", "qpos", "qrot", "qcdage", "misc"):
        g, w = np.asarray(got[k])[active], np.asarray(want[k])[active]
        if k in ("rot", "qrot"):
            same = (g.view(np.int64) == w.view(np.int64)) | ((g == 0) & (w == 0))
        else:
            same = g == w
        if not same.all():
            bad = np.argwhere(~same)[0]
            raise AssertionError(f"{where}: field {k} differs at {bad}: got {g[tuple(bad)]} want {w[tuple(bad)]}")


def compare_obs(obs, want_obs, active, where, tol=OBS_TOL):
    """obs: [2,E,12] (any float dtype); want_obs: [E,2,12] fp64 from the reference."""
    o = np.transpose(np.asarray(obs, dtype=np.float64), (1, 0, 2))[active]
    w = want_obs[active]
    # feature 11 (future collision flag) must match exactly
    if not (o[..., 11] == w[..., 11]).all():
        bad = np.argwhere(o[..., 11] != w[..., 11])[0]
        raise AssertionError(f"{where}: future-collision flag differs at {bad}")
    err = np.abs(o - w) / np.maximum(1.0, np.abs(w))
    if not (err <= tol).all():
        bad = np.unravel_index(np.argmax(err), err.shape)
        raise AssertionError(f"{where}: obs err {err[bad]:.3g} at {bad}: got {o[bad]!r} want {w[bad]!r}")


def compare_reward(rew, want_rew, active, where, tol=OBS_TOL):
    r = np.transpose(np.asarray(rew, dtype=np.float64), (1, 0))[active]
    w = want_rew[active]
    err = np.abs(r - w) / np.maximum(1.0, np.abs(w))
    if not (err <= tol).all():
        bad = np.unravel_index(np.argmax(err), err.shape)
        raise AssertionError(f"{where}: reward err {err[bad]:.3g} at {bad}: got {r[bad]} want {w[bad]}")


def replay(engine, d, obs_tol=OBS_TOL, check_every=1):
    """Drive `engine` through fixture `d` and check every tick.

    engine: object with load(state_arrays), arrays() -> state arrays (host numpy),
    step(actions[2,E,2], tick_limit) -> dict(obs[2,E,12], reward[2,E], done[E], winner[E]),
    move_direction(pid, speeds[E]), move_look(pid, angles[E]), shoot(pid, mask[E]),
    game_tick(), observe() -> (obs[2,E,12], reward[2,E]); optionally
    reward_simple() -> reward[2,E] of calculate_rewards_simple
    (SkillshotLearner.py:590-603) on the current state, held to the fixture's
    `reward_simple` series (the reference's own values) at every checked tick.
    Returns the number of env-ticks compared.
    """
    E = d["pos"].shape[0]
    n_steps = d["n_steps"]
    T = int(n_steps.max())
    engine.load(state_at(d, 0))
    obs0, rew0 = engine.observe()
    act0 = np.ones(E, bool)
    compare_obs(obs0, d["obs"][:, 0], act0, "t=0", obs_tol)
    compare_reward(rew0, d["reward"][:, 0], act0, "t=0", obs_tol)
    simple = hasattr(engine, "reward_simple") and "reward_simple" in d
    if simple:
        compare_reward(engine.reward_simple(), d["reward_simple"][:, 0], act0, "simple t=0", obs_tol)
    protocol = str(d["protocol"])
    compared = 0
    for t in range(T):
        a = np.ascontiguousarray(np.transpose(d["actions"][:, t], (1, 0, 2)))  # [2,E,2]
        if protocol == "learner":
            out = engine.step(a, int(d["tick_limit"]))
            obs, rew = out["obs"], out["reward"]
        else:
            for pid in (1, 2):
                engine.move_direction(pid, a[pid - 1, :, 0].astype(np.float64))
                engine.move_look(pid, a[pid - 1, :, 1].astype(np.float64))
                engine.shoot(pid, d["shoot"][:, t, pid - 1])
            engine.game_tick()
            obs, rew = engine.observe()
        active = n_steps >= t + 1
        if (t + 1) % check_every == 0 or t + 1 == T:
            compare_state(engine.arrays(), state_at(d, t + 1), active, f"{d['scenario']} t={t + 1}")
            compare_obs(obs, d["obs"][:, t + 1], active, f"{d['scenario']} t={t + 1}", obs_tol)
            compare_reward(rew, d["reward"][:, t + 1], active, f"{d['scenario']} t={t + 1}", obs_tol)
            if simple:
                compare_reward(engine.reward_simple(), d["reward_simple"][:, t + 1], active,
                               f"{d['scenario']} simple t={t + 1}", obs_tol)
            if protocol == "learner":
                live = d["live"][:, t + 1].astype(bool)
                ticks = d["ticks"][:, t + 1]
                want_done = (~live) | (ticks >= int(d["tick_limit"]))
                assert (out["done"][active].astype(bool) == want_done[active]).all(), f"done t={t + 1}"
                assert (out["winner"][active] == d["winner"][:, t + 1][active]).all(), f"winner t={t + 1}"
        compared += int(active.sum())
    return compared
