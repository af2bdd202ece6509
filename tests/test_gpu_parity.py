"""GPU parity: the HIP engine (libskillshot, through the C ABI) against the
reference golden vectors and the CPU oracle.

Bar: bit-exact on every state field (positions, fp64
rotations, projectile state, ticks, live, winner) and on done/winner;
obs/reward within 1e-5 relative to max(1,|ref|); the future-collision flag
(obs[11]) exact.
"""
import numpy as np
import pytest
import torch

import golden_replay as gr

pytestmark = pytest.mark.gpu

OBS_TOL = 1e-5


@pytest.fixture(scope="module")
def ssa():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import skillshot_learning_amd as m
    m.load_library()
    return m


def to_np(arrs):
    return {k: (v.cpu().numpy() if torch.is_tensor(v) else v) for k, v in arrs.items()}


class GpuEngine:
    """Adapter: golden_replay's engine protocol over VecSkillshotGame."""

    def __init__(self, ssa, n, **kw):
        self.g = ssa.VecSkillshotGame(n, **kw)

    def load(self, arrays):
        self.g.load_state_dict(arrays)

    def arrays(self):
        torch.cuda.synchronize()
        d = self.g.state_dict()
        d.pop("step_counter")
        return d

    def step(self, actions, tick_limit):
        self.g.tick_limit = tick_limit
        out = self.g.step(torch.as_tensor(actions).cuda(), obs=True, auto_reset=False)
        return to_np(out)

    def move_direction(self, pid, v):
        self.g.move_direction(pid, torch.as_tensor(v).cuda())

    def move_look(self, pid, v):
        self.g.move_look(pid, torch.as_tensor(v).cuda())

    def shoot(self, pid, mask):
        self.g.shoot(pid, torch.as_tensor(mask).cuda())

    def game_tick(self):
        self.g.game_tick()

    def observe(self):
        o, r = self.g.observe()
        return o.cpu().numpy(), r.cpu().numpy()

    def reward_simple(self):
        return self.g.observe(reward="simple")[1].cpu().numpy()


@pytest.fixture(params=[0, 1, 2], ids=["lane_per_env", "player_split", "fp32_fast"])
def step_variant(request, monkeypatch):
    """Every fused-step kernel (k_step, k_step_split, k_step_fast) must meet the same bar."""
    monkeypatch.setenv("SK_STEP_VARIANT", str(request.param))
    return request.param


@pytest.mark.parametrize("name", gr.fixture_names())
def test_golden_fixture(ssa, name, step_variant):
    d = gr.load(name)
    n = gr.replay(GpuEngine(ssa, d["pos"].shape[0]), d, obs_tol=OBS_TOL)
    assert n == int(d["n_steps"].sum())


def _random_state(oracle_mod, n, seed):
    s = oracle_mod.OracleState(n, seed=seed)
    s.reset(random_positions=True)
    return s


def _assert_state_equal(got, want, where):
    for k in want:
        g, w = np.asarray(got[k]), np.asarray(want[k])
        if k in ("rot", "qrot"):
            same = (g.view(np.int64) == w.view(np.int64)) | ((g == 0) & (w == 0))
        else:
            same = g == w
        if not same.all():
            bad = np.argwhere(~same)
            raise AssertionError(f"{where}: {k} differs in {len(bad)} entries, first {bad[0]}: "
                                 f"{g[tuple(bad[0])]} vs {w[tuple(bad[0])]}")


def test_fused_step_matches_oracle_random_policy(ssa, oracle_mod, step_variant):
    """8192 envs x 2500 ticks, random policy, random auto-reset (the learner
    protocol of configs 2/3): state bit-exact every 100 ticks, obs/reward/done/
    winner compared on sampled ticks, counters equal."""
    n, T = 8192, 2500
    ref = _random_state(oracle_mod, n, seed=42)
    g = ssa.VecSkillshotGame(n, seed=42, tick_limit=2000)
    g.load_state_dict(ref.arrays())
    g.step_counter = ref.step_counter
    g.clear_counters()
    checked = 0
    for t in range(T):
        acts = g.gen_random_actions(1)[0]
        ra = ref.gen_random_actions(1)[0]
        want_obs = (t % 97 == 0) or t == T - 1
        out = g.step(acts, obs=want_obs, auto_reset=True, reset_obs=want_obs)
        wo = ref.step(ra, tick_limit=2000, auto_reset=True, random_positions=True, want_obs=want_obs,
                      want_reset_obs=want_obs)
        if want_obs or t % 100 == 0:
            torch.cuda.synchronize()
            assert np.array_equal(acts.cpu().numpy(), ra), f"actions t={t}"
            assert np.array_equal(out["done"].cpu().numpy(), wo["done"]), f"done t={t}"
            assert np.array_equal(out["winner"].cpu().numpy(), wo["winner"]), f"winner t={t}"
            st = g.state_dict()
            st.pop("step_counter")
            _assert_state_equal(st, ref.arrays(), f"t={t}")
        if want_obs:
            o = out["obs"].cpu().numpy().astype(np.float64)
            err = np.abs(o - wo["obs"]) / np.maximum(1.0, np.abs(wo["obs"]))
            assert err.max() <= OBS_TOL, (t, err.max())
            assert np.array_equal(o[..., 11], wo["obs"][..., 11])
            r = out["reward"].cpu().numpy().astype(np.float64)
            assert (np.abs(r - wo["reward"]) / np.maximum(1.0, np.abs(wo["reward"]))).max() <= OBS_TOL
            orr = out["obs_reset"].cpu().numpy().astype(np.float64)
            assert (np.abs(orr - wo["obs_reset"]) / np.maximum(1.0, np.abs(wo["obs_reset"]))).max() <= OBS_TOL
            checked += 1
    c = g.counters()
    assert [c["dones"], c["hits_p1"], c["hits_p2"], c["ticks_sum"]] == [int(x) for x in ref.counters]
    assert c["dones"] > 1000 and c["hits_p1"] > 0 and c["hits_p2"] > 0
    assert checked > 10


@pytest.mark.parametrize("n,T", [(65536, 600), (1000, 4100)])
def test_rollout_random_matches_oracle(ssa, oracle_mod, n, T):
    """The multi-tick register-resident random-policy kernel (bench path) is
    bit-identical to the oracle's rollout, including ragged N (not a multiple
    of the 256-lane workgroup) and episodes crossing the 2000-tick limit."""
    ref = _random_state(oracle_mod, n, seed=7)
    g = ssa.VecSkillshotGame(n, seed=7, tick_limit=2000)
    g.load_state_dict(ref.arrays())
    g.step_counter = ref.step_counter
    g.clear_counters()
    done_ticks = 0
    for chunk in (1, T // 3, T - 1 - T // 3):
        g.rollout_random(chunk)
        ref.rollout_random(chunk, tick_limit=2000)
        done_ticks += chunk
        torch.cuda.synchronize()
        st = g.state_dict()
        assert st.pop("step_counter") == ref.step_counter
        _assert_state_equal(st, ref.arrays(), f"after {done_ticks} ticks")
    c = g.counters()
    assert [c["dones"], c["hits_p1"], c["hits_p2"], c["ticks_sum"]] == [int(x) for x in ref.counters]


def test_rollout_equals_stepwise_on_gpu(ssa, step_variant):
    """rollout_random(T) == T x (gen_random_actions + fused step) on device."""
    n, T = 3000, 300
    a = ssa.VecSkillshotGame(n, seed=3, tick_limit=120)
    a.reset(random_positions=True)
    b = ssa.VecSkillshotGame(n, seed=3, tick_limit=120)
    b.load_state_dict(a.state_dict())
    a.rollout_random(T)
    for _ in range(T):
        b.step(b.gen_random_actions(1)[0], obs=False, auto_reset=True)
    sa, sb = a.state_dict(), b.state_dict()
    for k in sa:
        assert np.array_equal(np.asarray(sa[k]), np.asarray(sb[k])), k
    assert a.counters() == b.counters()


def test_sharding_invariance(ssa):
    """Envs are keyed by GLOBAL id: two half-size shards (env_offset) equal one
    full run, the multi-GPU decomposition of SURVEY.md §8(e)."""
    n, T = 4096, 500
    full = ssa.VecSkillshotGame(n, seed=11, tick_limit=300)
    full.reset(random_positions=True)
    lo = ssa.VecSkillshotGame(n // 2, seed=11, env_offset=0, tick_limit=300)
    hi = ssa.VecSkillshotGame(n // 2, seed=11, env_offset=n // 2, tick_limit=300)
    lo.reset(random_positions=True)
    hi.reset(random_positions=True)
    full.rollout_random(T)
    lo.rollout_random(T)
    hi.rollout_random(T)
    f, a, b = full.state_dict(), lo.state_dict(), hi.state_dict()
    for k in f:
        if k == "step_counter":
            continue
        assert np.array_equal(f[k], np.concatenate([a[k], b[k]])), k


def test_features_match_oracle(ssa, oracle_mod):
    n = 20000
    ref = _random_state(oracle_mod, n, seed=5)
    # advance to get valid projectiles / varied rotations
    ref.rollout_random(37, tick_limit=2000)
    g = ssa.VecSkillshotGame(n)
    g.load_state_dict(ref.arrays())
    f = g.features().cpu().numpy()
    w = ref.features()
    # exact columns: x_dir, positions, rotation, cooldown, age, valid, future collision
    exact = [1, 4, 5, 6, 7, 9, 11, 12, 13, 14, 15, 17]
    assert np.array_equal(f[..., exact], w[..., exact])
    err = np.abs(f - w) / np.maximum(1.0, np.abs(w))
    assert err.max() <= 1e-12, err.max()


def test_per_method_ops_match_oracle(ssa, oracle_mod):
    """Discrete keyboard moves, masked shoot/reset, look and direction with
    per-env and scalar arguments, reward 'simple'."""
    n = 5000
    rng = np.random.default_rng(0)
    ref = _random_state(oracle_mod, n, seed=8)
    g = ssa.VecSkillshotGame(n, seed=8)
    g.load_state_dict(ref.arrays())
    g.step_counter = ref.step_counter
    for t in range(200):
        pid = 1 + (t % 2)
        sp = rng.uniform(-1.5, 1.5, n)
        ang = rng.uniform(-1.5, 1.5, n)
        mask = (rng.random(n) < 0.3).astype(np.uint8)
        kind = int(rng.integers(0, 4))
        g.move_direction(pid, torch.as_tensor(sp).cuda())
        ref.move_direction(pid, sp)
        g.move_look(pid, 0.125 if t % 5 == 0 else torch.as_tensor(ang).cuda())
        ref.move_look(pid, 0.125 if t % 5 == 0 else ang)
        g.move_discrete(pid, kind, torch.as_tensor(mask).cuda())
        ref.move_discrete(pid, kind, mask)
        if t % 3 == 0:
            g.shoot(pid, torch.as_tensor(1 - mask).cuda())
            ref.shoot(pid, 1 - mask)
        g.game_tick()
        ref.game_tick()
        if t % 50 == 49:
            rmask = (rng.random(n) < 0.1).astype(np.uint8)
            g.reset(torch.as_tensor(rmask).cuda(), random_positions=True)
            ref.reset(rmask, random_positions=True)
    torch.cuda.synchronize()
    st = g.state_dict()
    assert st.pop("step_counter") == ref.step_counter
    _assert_state_equal(st, ref.arrays(), "per-method")
    o, r = g.observe(reward="simple")
    wo, wr = ref.observe(reward_kind=1)
    assert (np.abs(o.cpu().numpy() - wo) / np.maximum(1, np.abs(wo))).max() <= OBS_TOL
    assert (np.abs(r.cpu().numpy() - wr) / np.maximum(1, np.abs(wr))).max() <= OBS_TOL


def test_large_batch_invariants(ssa):
    """Size-independent properties at the bench size (65,536 envs, config 2):
    bounds, tick limit, cooldown range under the always-shoot protocol, and
    counter consistency."""
    n = 65536
    g = ssa.VecSkillshotGame(n, seed=1, tick_limit=2000)
    g.reset(random_positions=True)
    g.clear_counters()
    g.rollout_random(3000)
    torch.cuda.synchronize()
    pos = g.pos.cpu().numpy()
    assert pos.min() >= 0 and pos.max() <= 245
    assert int(g.ticks.max()) <= 2000 and int(g.ticks.min()) >= 0
    cd = g.qcdage[:, [0, 2]].cpu().numpy()
    assert cd.min() >= 0 and cd.max() <= 15
    c = g.counters()
    assert c["dones"] >= c["hits_p1"] + c["hits_p2"]
    assert c["dones"] > n // 2
    # random policy: hits split about evenly between ids
    frac = c["hits_p1"] / max(1, c["hits_p1"] + c["hits_p2"])
    assert 0.4 < frac < 0.6
    mean_len = c["ticks_sum"] / c["dones"]
    assert 500 < mean_len < 1800


def test_errors_are_loud(ssa):
    g = ssa.VecSkillshotGame(64)
    with pytest.raises(ValueError):
        g.step(torch.zeros(2, 63, 2, device="cuda"))
    with pytest.raises(ssa.SkillshotError):
        g.move_direction(3, 0.5)


@pytest.mark.parametrize("name", [n for n in gr.fixture_names() if "reward_full" in gr.load(n)])
def test_full_reward_on_engine_features(ssa, name):
    """F3: calculate_rewards (SkillshotLearner.py:605-661) on the GPU, its
    inputs gathered from the HIP engine's get_state() features while the
    fixture's actions are replayed, against the reference's own output.  The
    engine's distances are correctly rounded sqrt, the reference's are libm
    pow or numpy sqrt by coordinate type (see test_rewards_full_cpu), so the
    bar is 1e-12 absolute; raised games must match exactly."""
    from skillshot_learning_amd.learner import calculate_rewards_full
    d = gr.load(name)
    E, T = d["pos"].shape[0], int(d["n_steps"].max())
    g = ssa.VecSkillshotGame(E, tick_limit=int(d["tick_limit"]))
    g.load_state_dict(gr.state_at(d, 0))
    feats, wins = [], []
    for t in range(T):
        a = torch.as_tensor(np.ascontiguousarray(np.transpose(d["actions"][:, t], (1, 0, 2)))).cuda()
        out = g.step(a, obs=False, auto_reset=False)
        feats.append(g.features().clone())
        wins.append(out["winner"].long())
    f = torch.stack(feats)
    lengths = torch.as_tensor(d["n_steps"].astype(np.int64)).cuda()
    r, raised = calculate_rewards_full(f[..., 16], f[..., 17] != 0, f[..., 14].long(), torch.stack(wins), lengths)
    want = d["reward_full"]
    want_raised = np.isnan(want[:, 0, 0])
    assert np.array_equal(raised.cpu().numpy(), want_raised)
    got = r.permute(1, 0, 2).cpu().numpy()
    m = ~np.isnan(want)
    assert np.array_equal(np.isnan(got), ~m)
    assert np.abs(got[m] - want[m]).max() <= 1e-12


def _flag_mismatches_explained(state, got11, want11):
    """obs[11] differences from the oracle (glibc tan) must all be projectiles
    whose gradient glibc does not round correctly and whose flag the correctly
    rounded tan decides the device's way (csrc/sk_tan_cr.hpp)."""
    import math
    from cr_tan import cr_tan
    bad = np.argwhere(got11 != want11)
    for p, i in bad:
        qx, qy = (int(v) for v in state["qpos"][i, 2 * p:2 * p + 2])
        ox, oy = (int(v) for v in state["pos"][i, 2 * (1 - p):2 * (1 - p) + 2])
        x = -float(state["qrot"][i, p]) + math.pi / 2
        g = cr_tan(x)
        assert math.tan(x) != g, (p, i)
        yi = float(qy) - g * float(qx)
        fut = any(float(oy) <= g * float(X) + yi <= float(oy + 5) for X in (ox, ox + 5))
        assert bool(got11[p, i]) == fut, (p, i)
    return len(bad)


def test_collision_probes_match_reference(ssa):
    """A9 / A11 on the probe boards (tests/golden/make_probes.py: projectiles
    a few pixels from the opponent, aimed corner shots, pi/4 multiples): the
    HIP check_collision equals the reference's exactly; the get_state
    future-collision feature and obs[11] equal the decision under the correctly
    rounded gradient (future_cr), which differs from the reference's only where
    glibc's tan is not correctly rounded; the get_state gradient is the
    correctly rounded tan bit for bit."""
    d = gr.load("probes")
    n = d["pos"].shape[0]
    g = ssa.VecSkillshotGame(n)
    g.load_state_dict(gr.probe_state(d))
    f = g.features().cpu().numpy()
    assert np.array_equal(f[..., 8].view(np.int64), d["grad_cr"].view(np.int64))
    assert np.array_equal(f[..., 17].astype(np.uint8), d["future_cr"])
    o, _ = g.observe()
    assert np.array_equal(o[..., 11].cpu().numpy().T.astype(np.uint8), d["future_cr"])
    differ = d["future_cr"] != d["future"]
    assert not (differ & (d["glibc_is_cr"] != 0)).any()
    hit = g.check_collision().cpu().numpy()
    assert np.array_equal(hit, d["hit"])
    flags = g.state_dict()["misc"][:, 1].view(np.uint32)
    assert np.array_equal(((flags >> 16) & 0xFF) == 0, d["hit"] != 0)
    assert np.array_equal(flags >> 24, d["hit"])


def test_fused_step_on_probe_boards(ssa, oracle_mod, step_variant):
    """The fused learner step from the probe boards (16 seeded copies each,
    96000 envs): projectiles start next to the opponent so most steps end in
    a corner hit or a near miss; state bit-exact vs the oracle, obs[11] equal
    except flags explained by glibc's tan rounding (see above)."""
    d = gr.load("probes")
    base = gr.probe_state(d)
    reps = 16
    arrays = {k: np.concatenate([v] * reps) for k, v in base.items()}
    n = arrays["pos"].shape[0]
    ref = oracle_mod.OracleState(n, seed=3)
    ref.load(arrays)
    g = ssa.VecSkillshotGame(n, seed=3, tick_limit=2000)
    g.load_state_dict(arrays)
    g.step_counter = ref.step_counter
    hits = explained = 0
    for t in range(4):
        acts = g.gen_random_actions(1)[0]
        ra = ref.gen_random_actions(1)[0]
        out = g.step(acts, obs=True, auto_reset=False, reset_obs=True)
        wo = ref.step(ra, tick_limit=2000, auto_reset=False)
        torch.cuda.synchronize()
        # no restart: the next tick's obs are this tick's, flags (and their
        # correctly rounded redo on ambiguous lanes) included
        assert torch.equal(out["obs_reset"], out["obs"]), t
        assert np.array_equal(out["done"].cpu().numpy(), wo["done"]), t
        assert np.array_equal(out["winner"].cpu().numpy(), wo["winner"]), t
        st = g.state_dict()
        st.pop("step_counter")
        _assert_state_equal(st, ref.arrays(), f"probe step {t}")
        o = out["obs"].cpu().numpy().astype(np.float64)
        explained += _flag_mismatches_explained(ref.arrays(), o[..., 11], wo["obs"][..., 11])
        assert (np.abs(o - wo["obs"]) / np.maximum(1.0, np.abs(wo["obs"])))[..., :11].max() <= OBS_TOL
        hits += int((wo["winner"] != 0).sum())
    assert hits > 1000
    assert explained <= 64


def test_cpu_backend_equals_gpu_engine(ssa):
    """The two libskillshot backends on one workload: the CPU backend
    (device = -1, csrc/sk_host.cpp) and the gfx950 engine, same start, same
    random-policy actions, random auto-reset: state / done / winner bit-exact,
    obs within 1e-5 with the future-collision flag exact, counters equal."""
    n, T = 4096, 900
    g = ssa.VecSkillshotGame(n, seed=5, tick_limit=400)
    g.reset(random_positions=True)
    c = ssa.VecSkillshotGame(n, device="cpu", seed=5, tick_limit=400)
    c.load_state_dict(g.state_dict())
    g.clear_counters()
    c.clear_counters()
    for t in range(T):
        a = g.gen_random_actions(1)[0]
        want = t % 89 == 0
        og = g.step(a, obs=want, auto_reset=True, reset_obs=want)
        oc = c.step(a.cpu(), obs=want, auto_reset=True, reset_obs=want)
        if want:
            torch.cuda.synchronize()
            assert np.array_equal(og["done"].cpu().numpy(), oc["done"].numpy()), t
            assert np.array_equal(og["winner"].cpu().numpy(), oc["winner"].numpy()), t
            for k in ("obs", "reward", "obs_reset"):
                x, y = og[k].cpu().numpy().astype(np.float64), oc[k].numpy().astype(np.float64)
                assert (np.abs(x - y) / np.maximum(1.0, np.abs(y))).max() <= OBS_TOL, (t, k)
            assert np.array_equal(og["obs"].cpu().numpy()[..., 11], oc["obs"].numpy()[..., 11]), t
    sg, sc = g.state_dict(), c.state_dict()
    _assert_state_equal({k: v for k, v in sg.items() if k != "step_counter"},
                        {k: v for k, v in sc.items() if k != "step_counter"}, "end")
    assert sg["step_counter"] == sc["step_counter"]
    assert g.counters() == c.counters()


@pytest.mark.parametrize("pol", [1, 0], ids=["write_through", "plain"])
@pytest.mark.parametrize("name", gr.fixture_names())
def test_golden_fixture_multi_obs(ssa, monkeypatch, name, pol):
    """The full-contract multi-tick kernel (sk_env_step_multi_obs, ABI 9): a
    learner-protocol fixture's whole trajectory in ONE launch (the action
    ring = the fixture's per-tick actions, one output slab per tick), every
    tick's obs / reward / done / winner and the final state against the
    reference's golden values, at the same bar as the one-tick kernels."""
    d = gr.load(name)
    if str(d["protocol"]) != "learner":
        pytest.skip("per-method protocol (no fused step)")
    monkeypatch.setenv("SK_MULTI_POLICY", str(pol))
    E = d["pos"].shape[0]
    n_steps = d["n_steps"]
    T = int(n_steps.max())
    g = ssa.VecSkillshotGame(E, tick_limit=int(d["tick_limit"]))
    g.load_state_dict(gr.state_at(d, 0))
    acts = np.ascontiguousarray(np.transpose(d["actions"][:, :T], (1, 2, 0, 3)))  # [T, 2, E, 2]
    out = g.step_multi_obs(torch.as_tensor(acts, dtype=torch.float32).cuda(), auto_reset=False)
    torch.cuda.synchronize()
    o = {k: v.cpu().numpy() for k, v in out.items()}
    for t in range(T):
        active = n_steps >= t + 1
        where = f"{d['scenario']} multi t={t + 1}"
        gr.compare_obs(o["obs"][t], d["obs"][:, t + 1], active, where, OBS_TOL)
        gr.compare_reward(o["reward"][t], d["reward"][:, t + 1], active, where, OBS_TOL)
        live = d["live"][:, t + 1].astype(bool)
        want_done = (~live) | (d["ticks"][:, t + 1] >= int(d["tick_limit"]))
        assert (o["done"][t][active].astype(bool) == want_done[active]).all(), where
        assert (o["winner"][t][active] == d["winner"][:, t + 1][active]).all(), where
    st = g.state_dict()
    st.pop("step_counter")
    gr.compare_state(st, gr.state_at(d, T), n_steps >= T, f"{d['scenario']} multi final")
