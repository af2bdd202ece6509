"""The pure-Python restatement (oracle/pyoracle.py) against the reference's
golden fixtures and against the C oracle: two independent CPU restatements
that must agree — bit-exact on state, done and winner; obs,
rewards and get_state values within 1e-12 (the reference's own `**`/pow
paths differ by an ulp between start modes, Appendix A rule 5)."""
import math

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import golden_replay as gr
from oracle.pyoracle import PyOracle

TOL = 1e-12


@pytest.mark.parametrize("name", gr.fixture_names())
def test_pyoracle_matches_reference(name):
    d = gr.load(name)
    n = gr.replay(PyOracle(d["pos"].shape[0]), d, obs_tol=TOL)
    assert n == int(d["n_steps"].sum())


def test_pyoracle_probe_boards():
    d = gr.load("probes")
    py = PyOracle(d["pos"].shape[0])
    py.load(gr.probe_state(d))
    f = py.features()
    assert np.array_equal(f[..., 17].astype(np.uint8), d["future"])
    hits = np.array([g.check_collision() for g in py.games], np.uint8)
    assert np.array_equal(hits, d["hit"])


@st.composite
def games(draw, n=4):
    coord = st.integers(0, 245)
    rots = st.one_of(st.floats(-40, 40, allow_nan=False), st.sampled_from([0.0, 0.25, -0.25, math.pi, -math.pi / 2]))
    arrs = dict(pos=np.zeros((n, 4), np.int32), rot=np.zeros((n, 2)), qpos=np.zeros((n, 4), np.int32),
                qrot=np.zeros((n, 2)), qcdage=np.zeros((n, 4), np.int32), misc=np.zeros((n, 2), np.int32))
    for i in range(n):
        p = [draw(coord) for _ in range(4)]
        arrs["pos"][i] = p
        arrs["qpos"][i] = [min(247, max(0, p[2 + k % 2] + draw(st.integers(-8, 8)))) for k in range(2)] + \
                          [min(247, max(0, p[k % 2] + draw(st.integers(-8, 8)))) for k in range(2)]
        arrs["rot"][i] = [draw(rots), draw(rots)]
        arrs["qrot"][i] = [draw(rots), draw(rots)]
        arrs["qcdage"][i] = [draw(st.integers(-30, 15)), draw(st.integers(0, 50)),
                             draw(st.integers(-30, 15)), draw(st.integers(0, 50))]
        qv = [draw(st.integers(0, 1)), draw(st.integers(0, 1))]
        flags = qv[0] | (qv[1] << 8) | (1 << 16)
        arrs["misc"][i] = [draw(st.integers(0, 1990)), flags]
    acts = np.array([[[draw(st.floats(-1.5, 1.5, width=32)), draw(st.floats(-1.5, 1.5, width=32))]
                      for _ in range(n)] for _ in range(2)], np.float32)
    return arrs, acts


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(games())
def test_pyoracle_equals_c_oracle_one_tick(oracle_mod, g):
    arrs, acts = g
    n = arrs["pos"].shape[0]
    c = oracle_mod.OracleState(n)
    c.load(arrs)
    py = PyOracle(n)
    py.load(arrs)
    fc, fp = c.features(), py.features()
    assert np.array_equal(fc[..., [1, 4, 5, 6, 7, 9, 11, 12, 13, 14, 15, 17]],
                          fp[..., [1, 4, 5, 6, 7, 9, 11, 12, 13, 14, 15, 17]])
    assert (np.abs(fc - fp) / np.maximum(1, np.abs(fp))).max() <= TOL
    wc = c.step(acts, tick_limit=2000, auto_reset=False)
    wp = py.step(acts, tick_limit=2000)
    for k, v in c.arrays().items():
        got = py.arrays()[k]
        same = (v.view(np.int64) == got.view(np.int64)) | ((v == 0) & (got == 0)) if v.dtype == np.float64 \
            else v == got
        assert same.all(), k
    assert np.array_equal(wc["done"], wp["done"]) and np.array_equal(wc["winner"], wp["winner"])
    assert (np.abs(wc["obs"] - wp["obs"]) / np.maximum(1, np.abs(wp["obs"]))).max() <= TOL
    assert (np.abs(wc["reward"] - wp["reward"]) / np.maximum(1, np.abs(wp["reward"]))).max() <= TOL
