"""libskillshot's CPU backend (device = -1, csrc/sk_host.cpp) through the C ABI
(VecSkillshotGame(device="cpu")): the reference golden fixtures, the oracle on
random-policy rollouts with random auto-reset, the multi-tick rollout, the
host-thread split and global-id sharding.

Bar: state, done and winner bit-exact; obs / rewards within
1e-5 relative to max(1, |ref|) with the future-collision flag exact.  This is
a product backend selected explicitly, not a fallback: VecSkillshotGame on
"cuda" still raises without a GPU."""
import numpy as np
import pytest
import torch

import golden_replay as gr

OBS_TOL = 1e-5


@pytest.fixture(scope="module")
def ssa():
    import skillshot_learning_amd as m
    m.load_library()
    return m


class CpuEngine:
    """golden_replay's engine protocol over VecSkillshotGame(device="cpu")"""

    def __init__(self, ssa, n):
        self.g = ssa.VecSkillshotGame(n, device="cpu")

    def load(self, arrays):
        self.g.load_state_dict(arrays)

    def arrays(self):
        d = self.g.state_dict()
        d.pop("step_counter")
        return d

    def step(self, actions, tick_limit):
        self.g.tick_limit = tick_limit
        out = self.g.step(torch.as_tensor(actions), obs=True, auto_reset=False)
        return {k: (v.numpy() if torch.is_tensor(v) else v) for k, v in out.items()}

    def move_direction(self, pid, v):
        self.g.move_direction(pid, torch.as_tensor(v))

    def move_look(self, pid, v):
        self.g.move_look(pid, torch.as_tensor(v))

    def shoot(self, pid, mask):
        self.g.shoot(pid, torch.as_tensor(mask))

    def game_tick(self):
        self.g.game_tick()

    def observe(self):
        o, r = self.g.observe()
        return o.numpy(), r.numpy()

    def reward_simple(self):
        return self.g.observe(reward="simple")[1].numpy()


@pytest.mark.parametrize("name", gr.fixture_names())
def test_cpu_backend_golden_fixture(ssa, name):
    d = gr.load(name)
    n = gr.replay(CpuEngine(ssa, d["pos"].shape[0]), d, obs_tol=OBS_TOL)
    assert n == int(d["n_steps"].sum())


def test_cpu_backend_features_match_reference_boards(ssa):
    """get_state numerics (SkillshotGame.py:136-166) on the reference boards:
    the CPU backend calls glibc's tan like CPython's math.tan, so it meets
    the reference to 1e-12 (the fixture's own rounding)."""
    d = gr.load("boards")
    k = d["pos"].shape[0]
    g = ssa.VecSkillshotGame(k, device="cpu")
    n = k
    z = np.zeros(n, np.int32)
    g.load_state_dict(dict(pos=d["pos"].reshape(n, 4), rot=d["rot"], qpos=d["qpos"].reshape(n, 4), qrot=d["qrot"],
                           qcdage=np.stack([d["qcd"][:, 0], d["qage"][:, 0], d["qcd"][:, 1], d["qage"][:, 1]], -1),
                           misc=np.stack([d["ticks"].astype(np.int32) + z,
                                          gr._flags(d["qvalid"], d["live"], d["winner"])], -1)))
    f = g.features().numpy()
    want = d["features"]
    assert (np.abs(f - want) <= 1e-12 * np.maximum(1.0, np.abs(want))).all()


def _assert_state_equal(got, want, where):
    for k in want:
        g, w = np.asarray(got[k]), np.asarray(want[k])
        same = ((g.view(np.int64) == w.view(np.int64)) | ((g == 0) & (w == 0))) if k in ("rot", "qrot") else g == w
        assert same.all(), f"{where}: {k} differs in {int((~same).sum())} entries"


def test_cpu_backend_matches_oracle_random_policy(ssa, oracle_mod):
    """2,048 games x 2,100 ticks of the random policy with random auto-reset
    (episodes cross the 2,000-tick cap): state bit-exact every 150 ticks,
    obs / reward / obs_reset / done / winner on sampled ticks, counters."""
    n, T = 2048, 2100
    ref = oracle_mod.OracleState(n, seed=42)
    ref.reset(random_positions=True)
    g = ssa.VecSkillshotGame(n, device="cpu", seed=42, tick_limit=2000)
    g.load_state_dict(ref.arrays())
    g.step_counter = ref.step_counter
    g.clear_counters()
    for t in range(T):
        acts = g.gen_random_actions(1)[0]
        ra = ref.gen_random_actions(1)[0]
        want = (t % 149 == 0) or t == T - 1
        out = g.step(acts, obs=want, auto_reset=True, reset_obs=want)
        wo = ref.step(ra, tick_limit=2000, auto_reset=True, random_positions=True, want_obs=want,
                      want_reset_obs=want)
        if want:
            assert np.array_equal(acts.numpy(), ra), t
            assert np.array_equal(out["done"].numpy(), wo["done"]) and np.array_equal(out["winner"].numpy(),
                                                                                      wo["winner"]), t
            st = g.state_dict()
            st.pop("step_counter")
            _assert_state_equal(st, ref.arrays(), f"t={t}")
            for k in ("obs", "reward", "obs_reset"):
                o = out[k].numpy().astype(np.float64)
                assert (np.abs(o - wo[k]) / np.maximum(1.0, np.abs(wo[k]))).max() <= OBS_TOL, (t, k)
            assert np.array_equal(out["obs"].numpy()[..., 11], wo["obs"][..., 11].astype(np.float32))
    c = g.counters()
    assert [c["dones"], c["hits_p1"], c["hits_p2"], c["ticks_sum"]] == [int(x) for x in ref.counters]
    assert c["dones"] > 500


def test_cpu_backend_rollout_equals_stepwise_and_threads(ssa, monkeypatch):
    """rollout_random(T) == T x (gen_random_actions + step); the host-thread
    split (SK_HOST_THREADS) does not change any bit"""
    n, T = 9000, 300
    a = ssa.VecSkillshotGame(n, device="cpu", seed=3, tick_limit=120)
    a.reset(random_positions=True)
    b = ssa.VecSkillshotGame(n, device="cpu", seed=3, tick_limit=120)
    b.load_state_dict(a.state_dict())
    monkeypatch.setenv("SK_HOST_THREADS", "1")
    c = ssa.VecSkillshotGame(n, device="cpu", seed=3, tick_limit=120)  # one thread (read at creation)
    c.load_state_dict(a.state_dict())
    a.rollout_random(T)
    c.rollout_random(T)
    for _ in range(T):
        b.step(b.gen_random_actions(1)[0], obs=False, auto_reset=True)
    sa, sb, sc = a.state_dict(), b.state_dict(), c.state_dict()
    for k in sa:
        assert np.array_equal(np.asarray(sa[k]), np.asarray(sb[k])), k
        assert np.array_equal(np.asarray(sa[k]), np.asarray(sc[k])), k
    assert a.counters() == b.counters() == c.counters()


def test_cpu_backend_sharding_invariance(ssa):
    """games keyed by GLOBAL id: two shards (env_offset) equal one run"""
    n, T = 4096, 400
    full = ssa.VecSkillshotGame(n, device="cpu", seed=11, tick_limit=300)
    lo = ssa.VecSkillshotGame(n // 2, device="cpu", seed=11, env_offset=0, tick_limit=300)
    hi = ssa.VecSkillshotGame(n // 2, device="cpu", seed=11, env_offset=n // 2, tick_limit=300)
    for g in (full, lo, hi):
        g.reset(random_positions=True)
        g.rollout_random(T)
    f, a, b = full.state_dict(), lo.state_dict(), hi.state_dict()
    for k in ("pos", "rot", "qpos", "qrot", "qcdage", "misc"):
        assert np.array_equal(f[k], np.concatenate([a[k], b[k]])), k


def test_cuda_request_without_gpu_raises(ssa):
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(ssa.SkillshotError):
        ssa.VecSkillshotGame(4, device="cuda")


def test_cpu_backend_step_insert_equals_step_then_add(ssa):
    """sk_env_step_insert on the CPU backend: the step's outputs and the ring
    rows of ReplayRing.add (torch path) after the same step, bit for bit,
    through wrap-around and restarts; total_copy (ABI 8) receives the new
    row count"""
    from skillshot_learning_amd.learner import ReplayRing
    n, cap = 37, 200
    a = ssa.VecSkillshotGame(n, device="cpu", seed=5, tick_limit=30)
    b = ssa.VecSkillshotGame(n, device="cpu", seed=5, tick_limit=30)
    ra, rb = ReplayRing(cap, "cpu", seed=1), ReplayRing(cap, "cpu", seed=1)
    oa, ob = a.observe()[0].clone(), b.observe()[0].clone()
    g = torch.Generator().manual_seed(2)
    for t in range(70):
        act = torch.rand((2, n, 2), generator=g) * 2.4 - 1.2
        copy = torch.full((1,), -1, dtype=torch.int64)
        x = a.step_insert(act, oa, ra, reset_obs=True, total_copy=copy if t % 2 else None)
        y = b.step(act, obs=True, reward="looking", auto_reset=True, reset_obs=True)
        rb.add(ob.reshape(-1, 12), act.reshape(-1, 2), y["reward"].reshape(-1), y["obs"].reshape(-1, 12), y["done"])
        for k in ("obs", "reward", "done", "winner", "obs_reset"):
            assert torch.equal(x[k], y[k]), (t, k)
        assert torch.equal(ra.buf, rb.buf), t
        assert int(ra.total_t) == int(rb.total_t) == ra.total == rb.total
        assert int(copy) == (ra.total if t % 2 else -1)
        oa, ob = x["obs_reset"], y["obs_reset"]
    assert a.counters()["dones"] > 0


def test_tick_form_selection():
    """TickGraph's tick form (learner.tick_form): sequential by default; the
    opt-in auto policy (streams
    from 16,384 games on one rank, fused below with the fp32 kernels, fused or
    sequential on several ranks) and the SK_TICK_OVERLAP overrides"""
    from skillshot_learning_amd.learner import tick_form

    # the default is the reference's order: the overlapped forms
    # are opt-in
    assert tick_form(4096, 256, 1 << 20, 1, False, True, True, True, True, env={}) == "sequential"
    assert tick_form(65536, 256, 1 << 20, 1, False, True, True, True, True, env={}) == "sequential"
    assert tick_form(4096, 256, 1 << 20, 1, True, True, True, True, True, env={}) == "sequential"

    def f(n, env=None, multi=False, f32=True, batch=256, cap=1 << 20, **kw):
        args = dict(updates_per_tick=1, fused=True, fused_act=True, sliced=True)
        args.update(kw)
        return tick_form(n, batch, cap, args["updates_per_tick"], multi, args["fused"], f32, args["fused_act"],
                         args["sliced"], env=dict({"SK_TICK_OVERLAP": "auto"}, **(env or {})))
    assert f(4096) == "fused" and f(65536) == "streams" and f(16384) == "streams"
    assert f(4096, f32=False) == "sequential" and f(65536, f32=False) == "streams"
    assert f(4096, multi=True) == "fused" and f(65536, multi=True) == "fused"
    assert f(4096, multi=True, f32=False) == "sequential"
    assert f(4098) == "sequential"                                  # N % 4 != 0: no fused launch
    assert f(4096, sliced=False) == "sequential"                    # batch past the sliced schedule
    assert f(4096, cap=4096) == "sequential"                        # ring too small beside an insert
    assert f(4096, updates_per_tick=2) == "sequential" and f(4096, fused=False) == "sequential"
    assert f(65536, env={"SK_TICK_OVERLAP": "0"}) == "sequential"
    assert f(4096, env={"SK_TICK_OVERLAP": "1"}) == "streams"
    assert f(4096, env={"SK_TICK_OVERLAP": "serial"}) == "serial"
    assert f(65536, env={"SK_TICK_OVERLAP": "fused"}) == "fused"
    assert f(4096, env={"SK_TICK_OVERLAP": "fused"}, f32=False) == "sequential"
    assert f(4096, env={"SK_FUSED_ACT": "0"}) == "sequential"
    assert f(65536, multi=True, env={"SK_TICK_OVERLAP": "1"}) == "sequential"
    assert f(4096, env={"SK_FUSED_REPLAY": "1"}) == "sequential"


def test_cpu_backend_step_multi_obs_equals_steps():
    """sk_env_step_multi_obs on the CPU backend (ABI 9): n_ticks sk_env_step
    calls with obs and reward, output slab (out0 + t) % out_slabs, bit for bit"""
    import skillshot_learning_amd as ssa
    n, T, R, S = 257, 90, 4, 6
    a = ssa.VecSkillshotGame(n, device="cpu", seed=3, tick_limit=40)
    a.reset(random_positions=True)
    b = ssa.VecSkillshotGame(n, device="cpu", seed=3, tick_limit=40)
    b.load_state_dict(a.state_dict())
    b.step_counter = a.step_counter
    acts = a.gen_random_actions(R)
    for reward in ("looking", "simple"):
        out = a.step_multi_obs(acts, n_ticks=T, slab0=3, out_slabs=S, out0=5, reward=reward)
        want = {}
        for t in range(T):
            o = b.step(acts[(3 + t) % R], obs=True, reward=reward, auto_reset=True)
            want[(5 + t) % S] = {k: o[k].clone() for k in ("obs", "reward", "done", "winner")}
        for s, w in want.items():
            for k, v in w.items():
                assert torch.equal(out[k][s], v.view(out[k][s].shape)), (reward, s, k)
        sa, sb = a.state_dict(), b.state_dict()
        for k in sa:
            assert np.array_equal(np.asarray(sa[k]), np.asarray(sb[k])), k
    assert a.counters() == b.counters() and a.counters()["dones"] > n
