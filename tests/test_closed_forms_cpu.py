"""Collision closed forms against the oracle's
procedural restatement and the reference's own outputs, on CPU.

* probes.npz (tests/golden/make_probes.py) holds 6000 boards written into the
  reference game with the projectile a few pixels from the opponent, and the
  reference's check_collision (SkillshotGame.py:58-94) / check_future_collision
  (SkillshotGame.py:96-113) results: the oracle and the closed forms must both
  reproduce them exactly.
* hypothesis then searches boards freely (positions, box-edge offsets, rotations
  including multiples of pi/4, aimed corner shots, validity) for any
  disagreement between the oracle's corner enumeration / x_dir-gated loop and
  the closed forms the HIP kernels evaluate:
    A9:  hit(p) = valid(q) and (qx+3 in [px, px+5] or qx in [px, px+5])
                           and (qy in [py, py+5] or qy-3 in [py, py+5]),
         player 1 tested first (the corner set is a product, so "some corner
         in the box" factors into one x and one y interval test);
    A11: valid and some X in {ox, ox+5} has oy <= g*X + (qy - g*qx) <= oy+5,
         g = tan(-r + pi/2), evaluated in fp64 in that operation order.
"""
import math

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import golden_replay as gr

PSIZE, QSIZE = 5, 3  # Player.py shape_size, Projectile.py shape_size


def hit_closed_form(pos, qpos, qvalid):
    """A9 on arrays: pos/qpos int [n,2,2], qvalid [n,2] -> u8 [n] id of the player hit."""
    out = np.zeros(pos.shape[0], np.uint8)
    for p in (1, 0):  # player 1 last so it overrides: first hit wins (SkillshotGame.py:79 break)
        q = 1 - p
        L, T = pos[:, p, 0], pos[:, p, 1]
        qx, qy = qpos[:, q, 0], qpos[:, q, 1]

        def inside(v, lo):
            return (lo <= v) & (v <= lo + PSIZE)

        hx = inside(qx + QSIZE, L) | inside(qx, L)
        hy = inside(qy, T) | inside(qy - QSIZE, T)
        hit = (qvalid[:, q] != 0) & hx & hy
        out[hit] = p + 1
    return out


def future_closed_form(qx, qy, qrot, valid, ox, oy):
    """A11 for one projectile (Python floats, libm tan as the reference's math.tan)."""
    if not valid:
        return 0
    g = math.tan(-qrot + math.pi / 2)
    yi = float(qy) - g * float(qx)
    for X in (ox, ox + PSIZE):
        v = g * float(X) + yi
        if float(oy) <= v <= float(oy + PSIZE):
            return 1
    return 0


def oracle_for(oracle_mod, arrays):
    n = arrays["pos"].shape[0]
    s = oracle_mod.OracleState(n)
    s.load(arrays)
    return s


def probe_arrays(d):
    return gr.probe_state(d)


def test_probes_fixture_has_boundary_cases():
    d = gr.load("probes")
    h = d["hit"]
    assert (h == 1).sum() > 100 and (h == 2).sum() > 100
    # both players hit at once: player 1 must take precedence in the fixture
    both = hit_closed_form(d["pos"], d["qpos"], d["qvalid"])
    assert np.array_equal(both, h)
    fut = d["future"]
    assert 0 < fut.sum() < fut.size


def test_oracle_collision_matches_reference_probes(oracle_mod):
    d = gr.load("probes")
    s = oracle_for(oracle_mod, probe_arrays(d))
    assert np.array_equal(s.check_collision(), d["hit"])
    misc = s.misc
    flags = misc[:, 1].view(np.uint32)
    live = (flags >> 16) & 0xFF
    winner = flags >> 24
    assert np.array_equal(live == 0, d["hit"] != 0)
    assert np.array_equal(winner, d["hit"])


def test_oracle_future_collision_matches_reference_probes(oracle_mod):
    d = gr.load("probes")
    s = oracle_for(oracle_mod, probe_arrays(d))
    f = s.features()
    assert np.array_equal(f[:, :, 17].astype(np.uint8), d["future"])


def test_closed_forms_match_reference_probes():
    d = gr.load("probes")
    assert np.array_equal(hit_closed_form(d["pos"], d["qpos"], d["qvalid"]), d["hit"])
    n = d["pos"].shape[0]
    got = np.array([[future_closed_form(d["qpos"][i, p, 0], d["qpos"][i, p, 1], d["qrot"][i, p],
                                        d["qvalid"][i, p], d["pos"][i, 1 - p, 0], d["pos"][i, 1 - p, 1])
                     for p in (0, 1)] for i in range(n)], np.uint8)
    assert np.array_equal(got, d["future"])


def test_probe_lines_reach_the_y_boundary():
    """The aimed probes put the projectile line within rounding of a box edge:
    the fp64 compare order matters on these (why the kernels keep it, no FMA)."""
    d = gr.load("probes")
    close = 0
    for i in range(d["pos"].shape[0]):
        for p in (0, 1):
            qx, qy = d["qpos"][i, p]
            ox, oy = d["pos"][i, 1 - p]
            g = math.tan(-d["qrot"][i, p] + math.pi / 2)
            yi = float(qy) - g * float(qx)
            for X in (ox, ox + PSIZE):
                v = g * float(X) + yi
                if min(abs(v - oy), abs(v - oy - PSIZE)) < 1e-9:
                    close += 1
    assert close >= 50, close


# ------------------------------------------------------------- hypothesis

coord = st.integers(min_value=0, max_value=245)
offset = st.integers(min_value=-9, max_value=9)
special_rot = st.sampled_from([k * math.pi / 4 for k in range(-16, 17)] + [0.0, -0.0, math.pi / 2 + 1e-12])
free_rot = st.floats(min_value=-30.0, max_value=30.0, allow_nan=False, allow_infinity=False)


@st.composite
def board(draw):
    pos = [[draw(coord), draw(coord)] for _ in range(2)]
    qpos, qrot = [], []
    for p in range(2):
        ox, oy = pos[1 - p]
        qx = min(247, max(0, ox + draw(offset)))
        qy = min(247, max(0, oy + draw(offset)))
        qpos.append([qx, qy])
        kind = draw(st.integers(0, 2))
        if kind == 0:
            r = draw(special_rot)
        elif kind == 1:
            r = draw(free_rot)
        else:  # aimed at an opponent corner (projectile moves by (-sin r, -cos r))
            cx, cy = ox + draw(st.sampled_from((0, PSIZE))), oy + draw(st.sampled_from((0, PSIZE)))
            r = math.atan2(-(cx - qx), -(cy - qy)) + draw(st.sampled_from((0.0, 1e-15, -1e-15, 2 * math.pi)))
        qrot.append(r)
    qvalid = [draw(st.integers(0, 1)) for _ in range(2)]
    return pos, qpos, qrot, qvalid


def _arrays(pos, qpos, qrot, qvalid):
    from oracle.oracle import pack_flags
    return dict(pos=np.array(pos, np.int32).reshape(1, 4), rot=np.zeros((1, 2)),
                qpos=np.array(qpos, np.int32).reshape(1, 4), qrot=np.array([qrot], np.float64),
                qcdage=np.zeros((1, 4), np.int32),
                misc=np.stack([np.zeros(1, np.int32), pack_flags(np.array([qvalid]), np.ones(1), np.zeros(1))], -1))


@settings(max_examples=3000, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(board())
def test_collision_closed_form_equals_oracle(oracle_mod, b):
    pos, qpos, qrot, qvalid = b
    s = oracle_for(oracle_mod, _arrays(pos, qpos, qrot, qvalid))
    want = hit_closed_form(np.array([pos]), np.array([qpos]), np.array([qvalid]))
    assert s.check_collision()[0] == want[0]


@settings(max_examples=3000, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(board())
def test_future_collision_closed_form_equals_oracle(oracle_mod, b):
    pos, qpos, qrot, qvalid = b
    s = oracle_for(oracle_mod, _arrays(pos, qpos, qrot, qvalid))
    f = s.features()[0, :, 17]
    for p in (0, 1):
        want = future_closed_form(qpos[p][0], qpos[p][1], qrot[p], qvalid[p], pos[1 - p][0], pos[1 - p][1])
        assert int(f[p]) == want, (p, b)


@pytest.mark.parametrize("seed", [0, 1])
def test_collision_closed_form_vectorised_sweep(oracle_mod, seed):
    """Every projectile offset in [-9, 9]^2 around the opponent, all validity
    combinations: the closed form and the oracle agree on the whole grid."""
    rng = np.random.default_rng(seed)
    offs = np.array([(dx, dy) for dx in range(-9, 10) for dy in range(-9, 10)])
    m = offs.shape[0] * 4
    pos = rng.integers(9, 237, size=(m, 2, 2)).astype(np.int32)
    qpos = np.zeros_like(pos)
    qvalid = np.array([(a, b) for a in (0, 1) for b in (0, 1)] * offs.shape[0], np.uint8)
    o = np.repeat(offs, 4, axis=0)
    qpos[:, 0] = pos[:, 1] + o
    qpos[:, 1] = pos[:, 0] + o[::-1]
    from oracle.oracle import pack_flags
    arrays = dict(pos=pos.reshape(m, 4), rot=np.zeros((m, 2)), qpos=qpos.reshape(m, 4), qrot=np.zeros((m, 2)),
                  qcdage=np.zeros((m, 4), np.int32),
                  misc=np.stack([np.zeros(m, np.int32), pack_flags(qvalid, np.ones(m), np.zeros(m))], -1))
    s = oracle_for(oracle_mod, arrays)
    assert np.array_equal(s.check_collision(), hit_closed_form(pos, qpos, qvalid))


def test_probe_flags_under_correctly_rounded_tan():
    """future_cr (the decision the HIP kernels are pinned to) differs from the
    reference's flag only on probes where glibc's tan is not correctly rounded."""
    from cr_tan import cr_tan
    d = gr.load("probes")
    x = -d["qrot"] + math.pi / 2
    for i in range(0, x.shape[0], 7):  # the stored CR gradients are what cr_tan gives
        for p in (0, 1):
            assert cr_tan(x[i, p]) == d["grad_cr"][i, p]
    glibc = np.vectorize(math.tan)(x)
    assert np.array_equal(glibc == d["grad_cr"], d["glibc_is_cr"] != 0)
    differ = d["future"] != d["future_cr"]
    assert not (differ & (d["glibc_is_cr"] != 0)).any()
    assert differ.sum() <= 3
    assert (d["glibc_is_cr"] == 0).sum() > 100
