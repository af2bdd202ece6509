"""The full-contract multi-tick kernel (sk_env_step_multi_obs, ABI 9;
VERDICT r03 item 5): n_ticks learner ticks with obs + reward in one launch
must equal n_ticks sk_env_step(obs, reward) launches bit for bit — every
tick's obs, reward, done and winner, the final state, the RNG step counter
and the episode counters — for both state ports, both rewards, ragged
batches, the 512-lane geometry (with the action-slab prefetch wave), output rings shorter than the launch, and
against the CPU backend (state bit-exact, obs within 1e-5: the CPU backend
computes obs with libm's tan, the kernels from the tick's sin/cos), and
launches of 1-3 ticks back to back."""
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


@pytest.mark.parametrize("reward", ["looking", "simple"])
@pytest.mark.parametrize("pol", [1, 0], ids=["write_through", "plain"])
@pytest.mark.parametrize("n,T,S", [(3000, 150, 150), (40000, 130, 7), (65536, 60, 4)])
def test_step_multi_obs_equals_stepwise(ssa, monkeypatch, reward, pol, n, T, S):
    R, slab0, out0, limit = 9, 4, 2, 50
    a, b = _pair(ssa, n, 17, limit, monkeypatch, pol)
    acts = a.gen_random_actions(R)
    a.clear_counters()
    b.clear_counters()
    out = a.step_multi_obs(acts, n_ticks=T, slab0=slab0, out_slabs=S, out0=out0, reward=reward)
    want = {}
    for t in range(T):
        o = b.step(acts[(slab0 + t) % R], obs=True, reward=reward, auto_reset=True)
        if t >= T - S:  # the ticks still held by the S-slab output ring
            want[(out0 + t) % S] = {k: o[k].clone() for k in ("obs", "reward", "done", "winner")}
    torch.cuda.synchronize()
    for s, w in want.items():
        for k, v in w.items():
            assert torch.equal(out[k][s], v.view(out[k][s].shape)), (s, k)
    _same_state(a, b)
    assert a.step_counter == b.step_counter
    ca, cb = a.counters(), b.counters()
    assert ca == cb and ca["dones"] > n  # limit 50 over >= 60 ticks: every game restarts


@pytest.mark.parametrize("T", [1, 2, 3])
def test_step_multi_obs_short_launches(ssa, monkeypatch, T):
    """launches of 1-3 ticks, back to back, into one output ring"""
    n, R, S = 5000, 7, 5
    a, b = _pair(ssa, n, 23, 4, monkeypatch, 1)
    acts = a.gen_random_actions(R)
    slab, so, want, out = 0, 0, {}, None
    for _ in range(4):
        out = a.step_multi_obs(acts, n_ticks=T, slab0=slab, out_slabs=S, out0=so, out=out)
        for t in range(T):
            o = b.step(acts[(slab + t) % R], obs=True, auto_reset=True)
            want[(so + t) % S] = {k: o[k].clone() for k in ("obs", "reward", "done", "winner")}
        torch.cuda.synchronize()
        for s, w in want.items():
            for k, v in w.items():
                assert torch.equal(out[k][s], v.view(out[k][s].shape)), (s, k)
        slab, so = (slab + T) % R, (so + T) % S
    _same_state(a, b)


@pytest.mark.parametrize("prefetch", ["0", "2", "4"])
def test_step_multi_obs_wide_and_ragged(ssa, monkeypatch, prefetch):
    """the 512-lane workgroups (SK_MULTI_BLOCK=512) and a ragged batch, with
    and without the action-slab prefetch wave (SK_MULTI_PREFETCH)"""
    monkeypatch.setenv("SK_MULTI_BLOCK", "512")
    monkeypatch.setenv("SK_MULTI_PREFETCH", prefetch)
    n, T, R = 131075, 40, 3
    a, b = _pair(ssa, n, 5, 30, monkeypatch, 1)
    acts = a.gen_random_actions(R)
    out = a.step_multi_obs(acts, n_ticks=T, out_slabs=2)
    last = None
    for t in range(T):
        last = b.step(acts[t % R], obs=True, auto_reset=True)
    torch.cuda.synchronize()
    s = (T - 1) % 2
    assert torch.equal(out["obs"][s], last["obs"]) and torch.equal(out["reward"][s], last["reward"])
    assert torch.equal(out["done"][s], last["done"])
    _same_state(a, b)


def test_step_multi_obs_cpu_backend(ssa, monkeypatch):
    monkeypatch.setenv("SK_MULTI_POLICY", "1")
    n, T, R = 4096, 120, 5
    g = ssa.VecSkillshotGame(n, seed=9, tick_limit=60)
    g.reset(random_positions=True)
    c = ssa.VecSkillshotGame(n, device="cpu", seed=9, tick_limit=60)
    c.load_state_dict(g.state_dict())
    c.step_counter = g.step_counter
    acts = g.gen_random_actions(R)
    g.clear_counters()
    c.clear_counters()
    og = g.step_multi_obs(acts, n_ticks=T, slab0=1)
    oc = c.step_multi_obs(acts.cpu(), n_ticks=T, slab0=1)
    torch.cuda.synchronize()
    for k in ("done", "winner"):
        assert np.array_equal(og[k].cpu().numpy(), oc[k].numpy()), k
    for k in ("obs", "reward"):
        x, y = og[k].cpu().double().numpy(), oc[k].double().numpy()
        err = np.abs(x - y) / np.maximum(1.0, np.abs(y))
        if k == "obs":  # the future-collision flag exact
            assert np.array_equal(x[..., 11], y[..., 11])
        assert err.max() <= 1e-5, (k, err.max())
    _same_state(g, c)
    assert g.counters() == c.counters()
