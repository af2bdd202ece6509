"""Pin the CPU oracle against the reference golden vectors (tests/golden/*.npz,
produced by running the reference game core: tests/golden/make_golden.py)."""
import numpy as np
import pytest

import golden_replay as gr


class OracleEngine:
    def __init__(self, oracle, n):
        self.s = oracle.OracleState(n)

    def load(self, arrays):
        self.s.load(arrays)

    def arrays(self):
        return self.s.arrays()

    def step(self, actions, tick_limit):
        return self.s.step(actions, tick_limit=tick_limit)

    def move_direction(self, pid, v):
        self.s.move_direction(pid, v)

    def move_look(self, pid, v):
        self.s.move_look(pid, v)

    def shoot(self, pid, mask):
        self.s.shoot(pid, mask)

    def game_tick(self):
        self.s.game_tick()

    def observe(self):
        return self.s.observe()

    def reward_simple(self):
        return self.s.observe(reward_kind=1)[1]


@pytest.mark.parametrize("name", gr.fixture_names())
def test_oracle_matches_reference(oracle_mod, name):
    d = gr.load(name)
    # the oracle uses libm pow like CPython: it must agree far tighter than the
    # engine's 1e-5 obs tolerance
    n = gr.replay(OracleEngine(oracle_mod, d["pos"].shape[0]), d, obs_tol=1e-12)
    assert n == int(d["n_steps"].sum())


def test_fixture_coverage():
    """The fixtures hold the edge cases SURVEY.md §4 asks for."""
    names = gr.fixture_names()
    both = gr.load("both_hit")
    # both players hit on the same tick -> P1 precedence (winner_id = 1, the hit player)
    ends = both["n_steps"]
    assert all(both["winner"][e, ends[e]] == 1 for e in range(len(ends)))
    raw = gr.load("raw")
    assert raw["qcd"].min() < -100  # cooldown unbounded below
    assert gr.load("negrot")["rot"].min() < -10
    ties = gr.load("ties")
    # y=50, rot 0, speed .5 -> 48.5 -> 48 (half-even); y=51 -> 49.5 -> 50
    assert ties["pos"][0, 1, 0, 1] == 48 and ties["pos"][1, 1, 0, 1] == 50
    clamp = gr.load("clamp")
    assert np.isinf(clamp["actions"]).any()
    fr = gr.load("fixed_random")
    assert (fr["n_steps"] == 2000).any() and (fr["winner"].max() > 0)
    assert "numpy_start" in names


def test_max_dist_constant(oracle_mod):
    # SkillshotLearner.py:43  (2 * (250 ** 2)) ** 0.5
    assert oracle_mod.max_dist() == (2 * (250 ** 2)) ** 0.5


def test_philox_known_answers(oracle_mod):
    """Random123 Philox4x32-10 known-answer vectors (kat_vectors)."""
    kat = [
        ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
        ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
        ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
         (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
    ]
    for ctr, key, want in kat:
        got = oracle_mod.philox4x32_10(ctr, key)
        assert tuple(int(x) for x in got) == want


def test_random_actions_range(oracle_mod):
    s = oracle_mod.OracleState(4096, seed=123)
    a = s.gen_random_actions(3)
    assert a.min() >= -1.0 and a.max() < 1.0
    assert abs(float(a.mean())) < 0.01
    # exactly representable: 2^-23 grid
    assert np.all(a * 2 ** 23 == np.round(a * 2 ** 23))


def test_random_reset_range(oracle_mod):
    s = oracle_mod.OracleState(20000, seed=5)
    s.reset(random_positions=True)
    assert s.pos.min() == 25 and s.pos.max() == 224
    assert (s.rot == 0).all() and (s.qcdage == 0).all()
    flags = oracle_mod.unpack_flags(s.misc[:, 1])
    assert (flags["live"] == 1).all() and (flags["winner"] == 0).all()


def test_rollout_equals_stepwise(oracle_mod):
    """rollout_random(T) == T x (gen_random_actions + step with random auto-reset)."""
    a = oracle_mod.OracleState(257, seed=9, env_offset=1000)
    a.reset(random_positions=True)
    b = a.copy()
    T = 700
    a.rollout_random(T, tick_limit=200)
    for _ in range(T):
        act = b.gen_random_actions(1)[0]
        b.step(act, tick_limit=200, auto_reset=True, random_positions=True, want_obs=False)
    for k, v in a.arrays().items():
        assert np.array_equal(v, b.arrays()[k]), k
    assert np.array_equal(a.counters, b.counters)
    assert a.counters[0] > 0
