"""k_step_multi (sk_env_step_multi): n_ticks step-only learner ticks in one
launch must equal n_ticks sk_env_step launches bit for bit — state, every
tick's done / winner, the RNG step counter and the episode counters — on a
ring of action slabs, for both state ports (plain / write-through), ragged
batches, the n >= 32,768 early restart draw, and against the CPU backend.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ssa():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import skillshot_learning_amd as m
    m.load_library()
    return m


@pytest.fixture(params=["0", "0e", "0p", "0q", "1", "1p", "1w"],
                ids=["lane_per_game_late_draw", "lane_per_game_early_draw", "lane_per_game_prefetch2", "lane_per_game_prefetch4",
                     "player_split", "player_split_prefetch2", "player_split_512"])
def split(request, monkeypatch):
    """every multi-tick geometry (k_step_multi, with or without the restart
    draw under the loads, with or without the prefetch wave; k_step_split_multi on 64-lane workgroups, and on
    512-lane ones with waves 4-7 staggered) meets the same bar"""
    monkeypatch.setenv("SK_MULTI_SPLIT", request.param[0])
    # the restart draw under the loads: on by default (round 6); "0" keeps the
    # draw in the restart branch
    monkeypatch.setenv("SK_MULTI_EARLY", "1" if request.param == "0e" else "0" if request.param == "0" else "-1")
    if request.param in ("0p", "0q", "1p"):  # the action-slab prefetch wave, 2 / 4 ticks ahead
        monkeypatch.setenv("SK_MULTI_PREFETCH", "4" if request.param == "0q" else "2")
    if request.param == "1w":
        monkeypatch.setenv("SK_MULTI_BLOCK", "512")
        monkeypatch.setenv("SK_MULTI_STAGGER", "2")
    return request.param


def _pair(ssa, n, seed, tick_limit, monkeypatch, pol):
    monkeypatch.setenv("SK_MULTI_POLICY", str(pol))
    a = ssa.VecSkillshotGame(n, seed=seed, tick_limit=tick_limit)
    a.reset(random_positions=True)
    b = ssa.VecSkillshotGame(n, seed=seed, tick_limit=tick_limit)
    b.load_state_dict(a.state_dict())
    b.step_counter = a.step_counter
    return a, b


def _same_state(x, y):
    sx, sy = x.state_dict(), y.state_dict()
    for k in sx:
        assert np.array_equal(np.asarray(sx[k]), np.asarray(sy[k])), k


@pytest.mark.parametrize("pol", [0, 1], ids=["plain", "write_through"])
@pytest.mark.parametrize("n", [3000, 40000])
def test_step_multi_equals_stepwise(ssa, monkeypatch, pol, n, split):
    T, R, slab0, limit = 300, 7, 3, 120
    a, b = _pair(ssa, n, 21, limit, monkeypatch, pol)
    acts = a.gen_random_actions(R)
    a.clear_counters()
    b.clear_counters()
    done, win = a.step_multi(acts, n_ticks=T, slab0=slab0, record=True)
    wd, ww = [], []
    for t in range(T):
        o = b.step(acts[(slab0 + t) % R], obs=False, auto_reset=True)
        wd.append(o["done"].clone())
        ww.append(o["winner"].clone())
    torch.cuda.synchronize()
    assert torch.equal(done, torch.stack(wd))
    assert torch.equal(win, torch.stack(ww))
    _same_state(a, b)
    ca, cb = a.counters(), b.counters()
    assert ca == cb and ca["dones"] > n  # limit 120 over 300 ticks: every game restarts


@pytest.mark.parametrize("pol", [0, 1], ids=["plain", "write_through"])
def test_step_multi_chunks_and_last_row(ssa, monkeypatch, pol, split):
    """Several launches of different lengths (slab0 carried over the ring)
    equal one; out_stride 0 leaves the last tick's done row."""
    n, R = 5000, 11
    a, b = _pair(ssa, n, 4, 2000, monkeypatch, pol)
    acts = a.gen_random_actions(R)
    s = 0
    for T in (1, 13, 40):
        d_last, w_last = a.step_multi(acts, n_ticks=T, slab0=s)
        s = (s + T) % R
    d_all, w_all = b.step_multi(acts, n_ticks=54, slab0=0, record=True)
    torch.cuda.synchronize()
    assert torch.equal(d_last, d_all[-1]) and torch.equal(w_last, w_all[-1])
    _same_state(a, b)
    assert a.counters() == b.counters()


def test_step_multi_cpu_backend_equals_gpu(ssa, monkeypatch, split):
    monkeypatch.setenv("SK_MULTI_POLICY", "1")
    n, T, R = 4096, 260, 5
    g = ssa.VecSkillshotGame(n, seed=9, tick_limit=100)
    g.reset(random_positions=True)
    c = ssa.VecSkillshotGame(n, device="cpu", seed=9, tick_limit=100)
    c.load_state_dict(g.state_dict())
    acts = g.gen_random_actions(R)
    g.clear_counters()
    c.clear_counters()
    dg, wg = g.step_multi(acts, n_ticks=T, slab0=2, record=True)
    dc, wc = c.step_multi(acts.cpu(), n_ticks=T, slab0=2, record=True)
    assert np.array_equal(dg.cpu().numpy(), dc.numpy())
    assert np.array_equal(wg.cpu().numpy(), wc.numpy())
    _same_state(g, c)
    assert g.counters() == c.counters()


@pytest.mark.parametrize("pack", ["1", "0"], ids=["packed", "exchange_form"])
def test_step_multi_states_outside_the_packed_range(ssa, monkeypatch, split, pack):
    """Games whose fields do not fit the packed resident form (cooldown far
    below -128, ages past 255, ticks past 65,535, a projectile 'valid' byte of
    3, positions off the board) keep their wave in the 88-B form; every other
    wave packs.  Both equal the stepwise kernels bit for bit."""
    monkeypatch.setenv("SK_MULTI_PACK", pack)
    n, T, R = 6000, 40, 3
    a, b = _pair(ssa, n, 33, 10 ** 6, monkeypatch, 1)
    st = a.state_dict()
    rng = np.random.default_rng(0)
    idx = rng.choice(n, 40, replace=False)
    st["qcdage"][idx[:10], 0] = -900
    st["qcdage"][idx[10:20], 3] = 100000
    st["misc"][idx[20:30], 0] = 70000
    st["misc"][idx[30:35], 1] = (st["misc"][idx[30:35], 1] & ~0xFF) | 3
    st["pos"][idx[35:40], 0] = 300
    for g in (a, b):
        g.load_state_dict(st)
    acts = a.gen_random_actions(R)
    done, win = a.step_multi(acts, n_ticks=T, record=True)
    for t in range(T):
        o = b.step(acts[t % R], obs=False, auto_reset=True)
        assert torch.equal(done[t], o["done"]) and torch.equal(win[t], o["winner"]), t
    _same_state(a, b)
