"""The learner at the reference's precision on the GPU (csrc/sk_learn32.hip,
fp32 operands on v_mfma_f32_32x32x2_f32) against the numpy fp64 restatement
of the reference's Keras arithmetic (oracle/keras_ref.py): critic and actor
gradients (SkillshotLearner.py:386-443), the bootstrap target, the actor
forward (:70-96) and its parameter noise (:245-281), and whole updates with
Keras Adam.

Bars: gradients within GRAD_REL = 1e-5 relative Frobenius per parameter
tensor; actor outputs within 1e-5 absolute; parameters after Adam steps within
PARAM_ABS = 1e-5 (1 % of one lr-sized Adam step).  Parity with Keras itself
stays unpinned (TensorFlow is absent)."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GRAD_REL = 1e-5
PARAM_ABS = 1e-5


@pytest.fixture(scope="module")
def mods():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import keras_ref
    from skillshot_learning_amd import learner
    return learner, keras_ref


@pytest.fixture(params=["0", "1"], ids=["one_launch", "sliced"])
def sched(request, monkeypatch):
    """both gradient schedules: one launch per step (16-row tiles per
    workgroup) and the sliced two-launch one (layer 2 over 8 workgroups per
    tile; automatic up to 512 rows) at every batch size"""
    monkeypatch.setenv("SK_SLICE32", request.param)
    return request.param


@pytest.fixture(params=["0", "1"], ids=["rows32", "rows16"])
def fwd(request, monkeypatch):
    """both actor forward kernels: 32-row tiles (large row counts) and
    16-row tiles (automatic below 32,768 rows)"""
    monkeypatch.setenv("SK_FWD16", request.param)
    return request.param


def _ddpg(learner, seed=0, scale=2.0, tau=None, gamma=0.0):
    d = learner.DDPG("cuda", seed=seed, tau=tau, gamma=gamma, fused_update=True, precision="fp32")
    with torch.no_grad():
        for m in (d.model_actor, d.model_critic):
            for l in (m.l1, m.l2, m.l3):
                l.weight.mul_(scale)
                l.bias.normal_(0, 0.1)
        if tau is not None:
            for dst, src in ((d.target_actor, d.model_actor), (d.target_critic, d.model_critic)):
                for pd, ps in zip(dst.parameters(), src.parameters()):
                    pd.copy_(ps * 1.1)
    return d


def _obs(rows, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.rand(rows, 12, device="cuda", generator=g) * torch.tensor(
        [1, 1, 1, 1, 9.8, 1, 1, 1, 1, 9.8, 1, 1.0], device="cuda")


def _np(t):
    return t.detach().double().cpu().numpy()


def _check_flat(flat, module, want, rel=GRAD_REL):
    off = 0
    for name, p in module.named_parameters():
        k = p.numel()
        got = flat[off:off + k].view_as(p).double().cpu().numpy()
        off += k
        err, den = np.linalg.norm(got - want[name]), np.linalg.norm(want[name])
        assert err <= rel * den + 1e-9, (name, err, den, err / max(den, 1e-30))


@pytest.mark.parametrize("rows", [1, 37, 256, 4096 + 17])
def test_critic_grad_f32_matches_keras(mods, sched, rows):
    learner, kr = mods
    d = _ddpg(learner, seed=1)
    s, a = _obs(rows, 1), torch.rand(rows, 2, device="cuda") * 2 - 1
    y = torch.randn(rows, device="cuda")
    mask = torch.zeros(rows, 256, dtype=torch.uint8, device="cuda")
    g = d._fused.grads("critic", s, a, y, mask_out=mask)
    torch.cuda.synchronize()
    if rows >= 256:
        assert abs(mask.float().mean().item() - 0.8) < 0.02
    want, _ = kr.critic_grads(kr.from_module(d.model_critic), _np(s), _np(a), _np(y), _np(mask))
    _check_flat(g, d.model_critic, want)


@pytest.mark.parametrize("rows", [37, 256, 4096 + 17])
def test_critic_grad_f32_bootstrap_matches_keras(mods, sched, rows):
    learner, kr = mods
    d = _ddpg(learner, seed=4, tau=0.05, gamma=0.9)
    s, a = _obs(rows, 2), torch.rand(rows, 2, device="cuda") * 2 - 1
    s2, r = _obs(rows, 3), torch.randn(rows, device="cuda")
    done = (torch.rand(rows, device="cuda") < 0.2).float()
    mask = torch.zeros(rows, 256, dtype=torch.uint8, device="cuda")
    g = d._fused.grads("critic", s, a, s2=s2, r=r, d=done, gamma=0.9, mask_out=mask)
    y = kr.target_y(kr.from_module(d.target_actor), kr.from_module(d.target_critic), _np(s2), _np(r), _np(done), 0.9)
    want, _ = kr.critic_grads(kr.from_module(d.model_critic), _np(s), _np(a), y, _np(mask))
    # the target adds an fp32 forward of two nets ahead of the gradient: 2e-5
    _check_flat(g, d.model_critic, want, rel=2e-5)


@pytest.mark.parametrize("rows", [1, 37, 256, 4096 + 17])
def test_actor_grad_f32_matches_keras(mods, sched, rows):
    learner, kr = mods
    d = _ddpg(learner, seed=2)
    s = _obs(rows, 4)
    g = d._fused.grads("actor", s)
    want, _ = kr.actor_grads(kr.from_module(d.model_actor), kr.from_module(d.model_critic), _np(s))
    _check_flat(g, d.model_actor, want)


def test_critic_grad_f32_split_rows_equal_whole(mods, sched):
    learner, _ = mods
    d = _ddpg(learner, seed=6)
    s, a, y = _obs(512, 5), torch.rand(512, 2, device="cuda") * 2 - 1, torch.randn(512, device="cuda")
    c0 = d._fused.calls.clone()
    whole = d._fused.grads("critic", s, a, y)
    tot = torch.zeros_like(whole)
    for lo, hi in ((0, 200), (200, 512)):
        d._fused.calls.copy_(c0)
        tot += d._fused.grads("critic", s[lo:hi], a[lo:hi], y[lo:hi], row_offset=lo, global_batch=512)
    assert (tot - whole).norm() <= 1e-6 * whole.norm()


@pytest.mark.parametrize("rows", [1, 33, 8192])
def test_actor_forward_f32_matches_keras(mods, fwd, rows):
    learner, kr = mods
    from skillshot_learning_amd.actor_kernel import ActorKernel32
    d = _ddpg(learner, seed=7)
    k = ActorKernel32(d.model_actor, seed=3)
    s = _obs(rows, 6)
    out = k(s)
    want, _ = kr.actor_forward(kr.from_module(d.model_actor), _np(s))
    assert np.abs(_np(out) - want).max() <= 1e-5


def test_actor_forward_f32_param_noise_distribution(mods, fwd):
    """model_act_param_noise (:245-281) per row: the kernel's outputs for one
    state repeated over 32,768 rows against explicit weight noise w (1 +
    0.5 N(0,1)) drawn per sample in fp64 (two-sample KS, moments); the device
    call counter advances once per launch and changes the draw."""
    learner, _ = mods
    from skillshot_learning_amd.actor_kernel import ActorKernel32
    d = _ddpg(learner, seed=8, scale=4.0)
    k = ActorKernel32(d.model_actor, seed=11)
    n = 32768
    x = _obs(1, 7).expand(n, 12).contiguous()
    got = k(x, noise_sd=0.5)
    got2 = k(x, noise_sd=0.5)
    torch.cuda.synchronize()
    assert int(k._ctr[0]) == 2 and not k._ctr[1:].any()  # every arrival slot back at 0
    assert not torch.equal(got, got2)
    g = torch.Generator(device="cuda").manual_seed(1)
    a = d.model_actor
    outs = []
    with torch.no_grad():
        for _ in range(n // 2048):
            h = x[:2048].double()
            for j, l in enumerate((a.l1, a.l2, a.l3)):
                W = l.weight.double().unsqueeze(0) * (1 + 0.5 * torch.randn((2048,) + tuple(l.weight.shape),
                                                                             device="cuda", generator=g,
                                                                             dtype=torch.float64))
                b = l.bias.double().unsqueeze(0) * (1 + 0.5 * torch.randn((2048,) + tuple(l.bias.shape),
                                                                           device="cuda", generator=g,
                                                                           dtype=torch.float64))
                h = torch.einsum("boi,bi->bo", W, h) + b
                h = torch.tanh(h) if j == 2 else torch.relu(h)
            outs.append(h)
    ex = torch.cat(outs).float().double().cpu()  # rounded like the kernel's: tanh saturates to exactly +-1 in fp32
    got = got.double().cpu()
    for j in range(2):
        m1, m2 = float(got[:, j].mean()), float(ex[:, j].mean())
        s1, s2 = float(got[:, j].std()), float(ex[:, j].std())
        assert abs(m1 - m2) < 5 * max(s1, s2) / math.sqrt(n) + 1e-3, (j, m1, m2)
        assert abs(s1 - s2) / max(s1, s2) < 0.04, (j, s1, s2)
        a_s, b_s = torch.sort(got[:, j]).values, torch.sort(ex[:, j]).values
        grid = torch.linspace(float(min(a_s[0], b_s[0])), float(max(a_s[-1], b_s[-1])), 400, dtype=torch.float64)
        fa = torch.searchsorted(a_s, grid).double() / n
        fb = torch.searchsorted(b_s, grid).double() / n
        assert float((fa - fb).abs().max()) < 1.95 * math.sqrt(2 / n) * 1.3


def test_f32_replay_updates_match_keras(mods, sched):
    """three fused fp32 replay updates (bootstrap target, critic step, actor
    step, Keras Adam, soft update) against the restatement step by step"""
    learner, kr = mods
    from skillshot_learning_amd import rng
    d = _ddpg(learner, seed=5, tau=0.05, gamma=0.9)
    A, C = kr.from_module(d.model_actor), kr.from_module(d.model_critic)
    TA, TC = kr.from_module(d.target_actor), kr.from_module(d.target_critic)
    oa, oc = kr.Adam(A), kr.Adam(C)
    for it in range(3):
        s, a = _obs(256, 20 + it), torch.rand(256, 2, device="cuda") * 2 - 1
        r, s2 = torch.randn(256, device="cuda"), _obs(256, 30 + it)
        dn = (torch.rand(256, device="cuda") < 0.2).float()
        keep = rng.dropout_keep(d.drop_seed, int(d.drop_calls), 0, 256).double().numpy()
        y = kr.target_y(TA, TC, _np(s2), _np(r), _np(dn), 0.9)
        gc, _ = kr.critic_grads(C, _np(s), _np(a), y, keep)
        C = oc.step(C, gc)
        ga, _ = kr.actor_grads(A, C, _np(s))
        A = oa.step(A, ga)
        TA, TC = kr.soft_update(TA, A, 0.05), kr.soft_update(TC, C, 0.05)
        d.update_batch(s, a, r, s2, dn)
        torch.cuda.synchronize()
        for mod, ref in ((d.model_critic, C), (d.model_actor, A), (d.target_critic, TC), (d.target_actor, TA)):
            for name, p in mod.named_parameters():
                err = np.abs(_np(p) - ref[name]).max()
                assert err <= PARAM_ABS, (it, name, err)


@pytest.mark.parametrize("overlap", ["0", "auto"])
def test_f32_learner_tick_graph(mods, overlap):
    """config 3 at the reference's precision: the captured learner tick with
    the fp32 kernels (actor forward with parameter noise, fused step, replay,
    fp32 critic / actor steps) runs, trains and stays finite, in the
    reference-order tick (default) and the opt-in overlapped (fused) one"""
    learner, _ = mods
    L = learner.SkillshotLearner(n_envs=4096, device="cuda", seed=23, exploration="param_noise", gamma=0.99,
                                 tau=0.005, replay_capacity=1 << 20, precision="fp32")
    assert L.ddpg._fused.f32
    tg = L.tick_graph(batch=256, ticks_per_graph=2, warmup=2, overlap=overlap)
    assert tg.mode == ("sequential" if overlap == "0" else "fused")
    w0 = [p.clone() for p in L.model_actor.parameters()]
    c0 = int(L.actor_kernel._ctr[0])
    tg.run(50)
    torch.cuda.synchronize()
    assert int(L.actor_kernel._ctr[0]) == c0 + 100  # one noise draw per tick
    assert all(bool(torch.isfinite(p).all()) for m in (L.model_actor, L.model_critic) for p in m.parameters())
    assert any((p - q).abs().max() > 0 for p, q in zip(L.model_actor.parameters(), w0))
    assert bool(torch.isfinite(tg.act).all()) and float(tg.act.abs().max()) <= 1.0


def test_actor_forward_f32_action_noise(mods, fwd):
    """model_act_action_noise (:229-243): the tanh outputs + N(0, 0.15) drawn
    in the kernel; the call counter advances per launch (fresh draws on every
    replay of a captured tick)"""
    learner, _ = mods
    from skillshot_learning_amd.actor_kernel import ActorKernel32
    d = _ddpg(learner, seed=9)
    k = ActorKernel32(d.model_actor, seed=5)
    x = _obs(65536, 9)
    clean = k(x)
    a1 = k(x, action_sd=0.15)
    a2 = k(x, action_sd=0.15)
    torch.cuda.synchronize()
    assert int(k._ctr[0]) == 2
    z = ((a1 - clean) / 0.15).double().cpu().flatten()
    assert abs(float(z.mean())) < 0.01 and abs(float(z.std()) - 1.0) < 0.01
    assert abs(float((z.abs() < 1).double().mean()) - 0.6827) < 0.01  # normal, not uniform
    assert not torch.equal(a1, a2)


def test_split_pack_follows_updates(mods):
    """the fp32 actor's split pack (sk_split.hpp) stays the pack of the
    current parameters: after fused updates (the actor's Adam launch rewrites
    it) it equals a fresh sk_actor_split_pack_f32 bit for bit, and a change
    made through torch is repacked at the next forward"""
    learner, kr = mods
    L = learner.SkillshotLearner(n_envs=512, device="cuda", seed=3, exploration="param_noise", gamma=0.9, tau=0.01,
                                 replay_capacity=1 << 14, precision="fp32")
    L.train_ticks(6, batch=128, warmup=128)
    torch.cuda.synchronize()
    k = L.actor_kernel
    got = k.pack.clone()
    k.refresh()
    torch.cuda.synchronize()
    assert torch.equal(got, k.pack)
    with torch.no_grad():
        L.model_actor.l2.weight.mul_(1.5)  # a torch-side change: the next call repacks
    s = _obs(8192, 2)
    out = k(s)
    want, _ = kr.actor_forward(kr.from_module(L.model_actor), _np(s))
    assert np.abs(_np(out) - want).max() <= 1e-5


@pytest.mark.parametrize("exploration,n", [("param_noise", 1024), ("action_noise", 1024), ("param_noise", 1028)])
def test_act_episode_equals_per_tick_loop(mods, monkeypatch, exploration, n):
    """sk_env_act_episode (the reference rule's episodes in one launch) against
    the per-tick loop (the 32-row actor forward, then sk_env_step without
    auto-reset, one launch each per tick): every played row's state, action
    and reward bit for bit, each game's length, and the final ticks / winner
    of every game at its end; the launch asks for more ticks than the limit
    allows, so every game ends before them, and the noise call number and
    the step counter advance by the loop's iterations, max(lengths), not by
    n_ticks (1,028 games: the last workgroup holds 4 of its 16)"""
    learner, _ = mods
    monkeypatch.setenv("SK_FWD16", "0")
    limit = 150
    L = learner.SkillshotLearner(n_envs=n, device="cuda", seed=5, exploration=exploration, tick_limit=limit,
                                 precision="fp32")
    g, k = L.game_environment, L.actor_kernel
    g.reset(random_positions=True)
    st0 = g.state_dict()
    obs = L.prepare_states().clone()
    c0 = int(k._ctr[0])
    sd = L.param_noise_sd if exploration == "param_noise" else 0.0
    asd = L.action_noise_sd if exploration == "action_noise" else 0.0
    step0 = g.step_counter
    ep = g.act_episode(k, obs, n_ticks=limit + 50, noise_sd=sd, action_sd=asd)
    torch.cuda.synchronize()
    got_len = ep["lengths"].long()
    T = int(got_len.max())
    assert T <= limit < limit + 50
    assert int(k._ctr[0]) == c0 + (T if sd or asd else 0)
    got_step = g.step_counter
    assert got_step == step0 + T
    end_ticks, end_winner = g.ticks.clone(), g.winner_id.clone()
    # the per-tick loop from the same start and call number
    g.load_state_dict(st0)
    k._ctr[0] = c0
    alive = torch.ones(n, dtype=torch.bool, device="cuda")
    length = torch.zeros(n, dtype=torch.long, device="cuda")
    want_ticks = torch.zeros(n, dtype=torch.int32, device="cuda")
    want_winner = torch.zeros(n, dtype=torch.uint8, device="cuda")
    s = obs
    for t in range(limit):
        a = k(s.reshape(-1, 12), noise_sd=sd, action_sd=asd).reshape(2, n, 2)
        out = g.step(a, obs=True, reward="looking", auto_reset=False)
        m = alive
        assert torch.equal(ep["states"][t][:, m], s[:, m]), t
        assert torch.equal(ep["actions"][t][:, m], a[:, m]), t
        assert torch.equal(ep["rewards"][t][:, m], out["reward"][:, m]), t
        assert torch.equal(ep["states"][t + 1][:, m], out["obs"][:, m]), t
        length += alive.long()
        newly = alive & out["done"].bool()
        want_ticks = torch.where(newly, g.ticks, want_ticks)
        want_winner = torch.where(newly, out["winner"], want_winner)
        alive = alive & ~out["done"].bool()
        s = out["obs"]
        if not bool(alive.any()):
            break
    assert torch.equal(got_len, length)
    assert torch.equal(end_ticks, want_ticks) and torch.equal(end_winner, want_winner)
    torch.cuda.synchronize()
    assert int(k._ctr[0]) == c0 + (T if sd or asd else 0) and g.step_counter == got_step  # the loop's advance
    assert int(got_len.max()) > 1 and int((got_len < limit).sum()) > 0  # both endings occur


@pytest.mark.parametrize("chunk", ["", "7"])
def test_model_train_on_device_equals_loop(mods, monkeypatch, chunk):
    """model_train with the episodes in one launch (default) and with the
    per-tick loop (SK_EPISODE_KERNEL=0): the same nets after two epochs, bit
    for bit (same rows in the same order, the same shuffle, the next epoch's
    restarts and noise from the same counters).  chunk "7": the episodes in
    launches of 7 ticks (SK_EPISODE_CHUNK), each continuing from the last;
    the final one ends short of its 7, i.e. every game ends before the
    launch's tick count"""
    learner, _ = mods
    monkeypatch.setenv("SK_FWD16", "0")
    if chunk:
        monkeypatch.setenv("SK_EPISODE_CHUNK", chunk)
    nets = []
    for flag in ("1", "0"):
        monkeypatch.setenv("SK_EPISODE_KERNEL", flag)
        L = learner.SkillshotLearner(n_envs=256, device="cuda", seed=9, tick_limit=60, precision="fp32")
        prog = L.model_train(2)
        torch.cuda.synchronize()
        nets.append((torch.cat([p.detach().flatten() for p in L.model_actor.parameters()]),
                     torch.cat([p.detach().flatten() for p in L.model_critic.parameters()]),
                     torch.stack(prog["epoch_ticks"]), torch.stack(prog["epoch_winner"])))
    for x, y in zip(*nets):
        assert torch.equal(x, y)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_models_fit_graph_chunks_equal_eager(mods, monkeypatch, precision):
    """models_fit's three-launch steps (SK_FIT_RESIDENT=0) with its
    minibatches replayed as captured chunks (default)
    against one eager launch set per minibatch (SK_FIT_GRAPH=0): the same
    nets and Adam moments bit for bit (3,000 rows: the first minibatch
    eager, two chunks of 64, the remainder and the partial last batch eager)"""
    learner, _ = mods
    monkeypatch.setenv("SK_FIT_RESIDENT", "0")
    g = torch.Generator(device="cuda").manual_seed(3)
    rows = 3000
    s = torch.rand(rows, 12, device="cuda", generator=g)
    a = torch.rand(rows, 2, device="cuda", generator=g) * 2 - 1
    r = torch.randn(rows, device="cuda", generator=g)
    out = []
    for flag in ("1", "0"):
        monkeypatch.setenv("SK_FIT_GRAPH", flag)
        d = learner.DDPG("cuda", seed=4, fused_update=True, precision=precision)
        d.models_fit(s, a, r)
        d.models_fit(s[:700], a[:700], r[:700])  # a second call reuses the captured graphs
        torch.cuda.synchronize()
        out.append([p.detach().clone() for m in (d.model_actor, d.model_critic) for p in m.parameters()] +
                   [d._fused.sa.m.clone(), d._fused.sc.v.clone()])
    for x, y in zip(*out):
        assert torch.equal(x, y)


def test_models_fit_graph_losses_private(mods, monkeypatch):
    """the captured models_fit chunks write their steps' losses into a buffer
    of their own: the eager steps' history (loss_hist, whose
    returned scalars stay valid for LOSS_HIST further steps) holds only the
    eager steps' losses.  1,200 rows at batch 16: 75 minibatches per pass =
    the first eager, one captured chunk of 64, ten eager"""
    learner, _ = mods
    g = torch.Generator(device="cuda").manual_seed(6)
    s = torch.rand(1200, 12, device="cuda", generator=g)
    a = torch.rand(1200, 2, device="cuda", generator=g) * 2 - 1
    r = torch.randn(1200, device="cuda", generator=g)
    monkeypatch.setenv("SK_FIT_RESIDENT", "0")  # the three-launch steps and their captured chunks
    d = learner.DDPG("cuda", seed=4, fused_update=True, precision="fp32")
    fu = d._fused
    d.models_fit(s, a, r)
    torch.cuda.synchronize()
    hist = fu.loss_hist.cpu()
    assert fu._li == [11, 11]
    assert bool((hist[:, :11] != 0).all()) and bool((hist[:, 11:] == 0).all())
    assert len(d._fit_graphs) == 2
    for (_, _, critic), v in d._fit_graphs.items():  # row 0: the critic steps' losses, row 1: the actor's
        k = 0 if critic else 1
        assert bool((v[4][k] != 0).all()) and bool((v[4][1 - k] == 0).all())


def _fit_rows(n, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    s = torch.rand(n, 12, device="cuda", generator=g) * torch.tensor(
        [1, 1, 1, 1, 9.8, 1, 1, 1, 1, 9.8, 1, 1.0], device="cuda")
    return s, torch.rand(n, 2, device="cuda", generator=g) * 2 - 1, torch.randn(n, device="cuda", generator=g) * 0.5


def _check_placement(fu, xcd):
    """the launch's placement report (timeout word 1, csrc/sk_fit.hip
    fit_placement): the default stride-8 grid lands on one XCD (2: plain
    exchange stores through its L2); the spread grid on several (1:
    write-through), or on one where the device is a single XCD"""
    place = int(fu.fit_timeout[1].item())
    assert place == 2 if xcd == "1" else place in (1, 2), place


@pytest.mark.parametrize("p,xcd", [("16", "0"), ("16", "1"), ("8", "1")])
def test_fit_critic_resident_equals_eager_and_keras(mods, monkeypatch, p, xcd):
    """models_fit's critic pass in resident launches (sk_fit_critic_f32,
    csrc/sk_fit.hip: the net split over 16 or 8 workgroups by layer-2 input
    columns, SK_FIT_P, two in-launch exchanges per step; on one XCD and
    spread over the XCDs, SK_FIT_XCD) against one three-launch
    critic_step per minibatch (sk_critic_grad_f32 + sk_adam_flat) and the
    fp64 Keras restatement, over 96 minibatch steps in two launches (64 +
    32): parameters within 1e-5, Adam moments, step counts, the Dropout call
    number and the per-step losses"""
    learner, kr = mods
    from skillshot_learning_amd import rng
    monkeypatch.setenv("SK_FIT_XCD", xcd)
    monkeypatch.setenv("SK_FIT_P", p)
    n = 96
    s, a, y = _fit_rows(16 * n, 7)
    dr = _ddpg(learner, seed=3, scale=2.0)
    de = _ddpg(learner, seed=3, scale=2.0)
    fr, fe = dr._fused, de._fused
    C0 = kr.from_module(de.model_critic)
    call0 = int(de.drop_calls)
    losses = torch.zeros(n, device="cuda")
    fr.FIT_STEPS_PER_LAUNCH = 64
    assert fr.fit_critic(s, a, y, losses=losses) == n
    fr.fit_check()
    _check_placement(fr, xcd)
    want_loss = []
    for k in range(n):
        sl = slice(16 * k, 16 * k + 16)
        want_loss.append(float(de.critic_step(s[sl], a[sl], y[sl])))
    torch.cuda.synchronize()
    assert int(dr.drop_calls) == int(de.drop_calls) == call0 + n
    assert torch.equal(fr.sc.steps, fe.sc.steps)
    got, want = fr.fc.double().cpu().numpy(), fe.fc.double().cpu().numpy()
    assert np.abs(got - want).max() <= PARAM_ABS, np.abs(got - want).max()
    for x, z in ((fr.sc.m, fe.sc.m), (fr.sc.v, fe.sc.v)):
        assert (x - z).abs().max().item() <= 1e-4 * z.abs().max().item()
    assert np.allclose(losses.cpu().numpy(), want_loss, rtol=1e-4, atol=1e-6)
    # the fp64 Keras restatement, step by step (Dropout keys of each step's call)
    C = C0
    oc = kr.Adam(C)
    sn, an, yn = _np(s), _np(a), _np(y)
    for k in range(n):
        sl = slice(16 * k, 16 * k + 16)
        keep = rng.dropout_keep(de.drop_seed, call0 + k, 0, 16).double().numpy()
        gc, _ = kr.critic_grads(C, sn[sl], an[sl], yn[sl], keep)
        C = oc.step(C, gc)
    ref = np.concatenate([C[name].reshape(-1) for name, _ in de.model_critic.named_parameters()])
    assert np.abs(got - ref).max() <= PARAM_ABS, np.abs(got - ref).max()


def test_fit_critic_launch_longer_than_step_size_table(mods):
    """one resident critic launch of 2,100 minibatch steps (past the
    2,048-step table of Adam step sizes each launch refills in LDS,
    csrc/sk_fit.hip alpha_fill) equals, bit for bit, the same pass cut into
    launches of 512 steps (no refill): nets, Adam moments and step counts,
    the Dropout call number.  (Against the three-launch chain a pass this long
    is not a parity bar: a pre-activation within the two summation orders'
    ~1e-7 of zero flips a relu somewhere in ~10^7 decisions and the two
    trajectories part, tools/diag_fit_long.py.)"""
    learner, _ = mods
    n = 2100
    s, a, y = _fit_rows(16 * n, 13)
    out = []
    for per in (4096, 512):
        d = _ddpg(learner, seed=6, scale=1.0)
        d._fused.FIT_STEPS_PER_LAUNCH = per
        assert d._fused.fit_critic(s, a, y) == n
        d._fused.fit_check()
        torch.cuda.synchronize()
        f = d._fused
        out.append((f.fc.clone(), f.sc.m.clone(), f.sc.v.clone(), f.sc.steps.clone(), int(d.drop_calls)))
    (c1, m1, v1, t1, k1), (c2, m2, v2, t2, k2) = out
    assert k1 == k2 and torch.equal(t1, t2)
    assert torch.equal(c1, c2) and torch.equal(m1, m2) and torch.equal(v1, v2)
    assert bool(torch.isfinite(c1).all())


def test_fit_placements_equal_bit_for_bit(mods, monkeypatch):
    """the exchange's two store flavours (plain stores through one XCD's L2,
    write-through stores spread over the XCDs) carry the same values in the
    same summation order: a 700-step critic pass and actor pass on each give
    the same nets, moments and losses bit for bit"""
    learner, _ = mods
    n = 700
    s, a, y = _fit_rows(16 * n, 17)
    out = []
    for xcd in ("1", "0"):
        monkeypatch.setenv("SK_FIT_XCD", xcd)
        d = _ddpg(learner, seed=8, scale=1.0)
        f = d._fused
        losses = torch.zeros(n, device="cuda")
        assert f.fit_critic(s, a, y, losses=losses) == n
        assert f.fit_actor(s) == n
        f.fit_check()
        _check_placement(f, xcd)
        torch.cuda.synchronize()
        out.append([f.fc.clone(), f.sc.m.clone(), f.sc.v.clone(), f.fa.clone(), f.sa.m.clone(), f.sa.v.clone(),
                    losses])
    for x, z in zip(*out):
        assert torch.equal(x, z)


def test_models_fit_resident_equals_three_launch(mods, monkeypatch):
    """models_fit with the resident critic pass (default) and with the
    three-launch steps (SK_FIT_RESIDENT=0): the same nets within 1e-5 after a
    pass over 1,613 rows (100 full minibatches and a partial one), and the
    same Dropout call number and Adam step counts"""
    learner, _ = mods
    s, a, y = _fit_rows(1613, 9)
    out = []
    for flag in ("1", "0"):
        monkeypatch.setenv("SK_FIT_RESIDENT", flag)
        d = learner.DDPG("cuda", seed=4, fused_update=True, precision="fp32")
        d.models_fit(s, a, y)
        torch.cuda.synchronize()
        out.append((d._fused.fc.clone(), d._fused.fa.clone(), int(d.drop_calls), d._fused.sc.steps.clone(),
                    d._fused.sa.steps.clone()))
    (c1, a1, k1, s1, t1), (c0, a0, k0, s0, t0) = out
    assert k1 == k0 and torch.equal(s1, s0) and torch.equal(t1, t0)
    assert (c1 - c0).abs().max().item() <= PARAM_ABS
    assert (a1 - a0).abs().max().item() <= PARAM_ABS


@pytest.mark.parametrize("p,xcd", [("16", "1"), ("16", "0"), ("8", "1")])
def test_fit_actor_resident_equals_eager_and_keras(mods, monkeypatch, p, xcd):
    """models_fit's actor pass in resident launches (sk_fit_actor_f32: the
    frozen critic's pre-activations computed up front, the actor split over
    16 or 8 workgroups by layer-2 input columns, two in-launch exchanges per
    step; on one XCD and spread) against one three-launch
    model_actor_fit_step per minibatch and the fp64 Keras restatement, over
    96 minibatch steps in two launches: parameters within 1e-5, Adam step
    counts equal, the critic untouched, the split pack rewritten"""
    learner, kr = mods
    monkeypatch.setenv("SK_FIT_P", p)
    monkeypatch.setenv("SK_FIT_XCD", xcd)
    n = 96
    s, _, _ = _fit_rows(16 * n, 11)
    dr = _ddpg(learner, seed=5, scale=2.0)
    de = _ddpg(learner, seed=5, scale=2.0)
    fr, fe = dr._fused, de._fused
    A0, C0 = kr.from_module(de.model_actor), kr.from_module(de.model_critic)
    crit0 = fr.fc.clone()
    from skillshot_learning_amd.actor_kernel import ActorKernel32
    k = ActorKernel32(dr.model_actor, seed=3)
    fr.split_pack = k.ensure_pack()
    fr.FIT_STEPS_PER_LAUNCH = 64
    assert fr.fit_actor(s) == n
    fr.fit_check()
    _check_placement(fr, xcd)
    for j in range(n):
        de.model_actor_fit_step(s[16 * j:16 * j + 16])
    torch.cuda.synchronize()
    assert torch.equal(fr.fc, crit0)
    assert torch.equal(fr.sa.steps, fe.sa.steps)
    got, want = fr.fa.double().cpu().numpy(), fe.fa.double().cpu().numpy()
    assert np.abs(got - want).max() <= PARAM_ABS, np.abs(got - want).max()
    A = A0
    oa = kr.Adam(A)
    sn = _np(s)
    for j in range(n):
        ga, _ = kr.actor_grads(A, C0, sn[16 * j:16 * j + 16])
        A = oa.step(A, ga)
    ref = np.concatenate([A[name].reshape(-1) for name, _ in de.model_actor.named_parameters()])
    assert np.abs(got - ref).max() <= PARAM_ABS, np.abs(got - ref).max()
    # the acting kernel reads the rewritten pack: its forward equals a fresh pack's
    x = _obs(64, 12)
    out = k(x)
    k2 = ActorKernel32(dr.model_actor, seed=3)
    assert torch.equal(out, k2(x))


def test_fit_step_counts_saturate_like_the_chain(mods):
    """Adam step counts past 2^24: the three-launch chain adds
    1.0f per step, which stops changing the count at 2^24; the resident
    launches store the same saturated count (and take their step sizes at
    it).  From 2^24 - 8, 32 critic and 32 actor steps: counts equal (2^24),
    nets within PARAM_ABS of the chain's"""
    learner, _ = mods
    n = 32
    s, a, y = _fit_rows(16 * n, 21)
    dr = _ddpg(learner, seed=9, scale=1.0)
    de = _ddpg(learner, seed=9, scale=1.0)
    t0 = float(2 ** 24 - 8)
    for d in (dr, de):
        d._fused.sc.steps.fill_(t0)
        d._fused.sa.steps.fill_(t0)
    fr, fe = dr._fused, de._fused
    assert fr.fit_critic(s, a, y) == n
    assert fr.fit_actor(s) == n
    fr.fit_check()
    for k in range(n):
        sl = slice(16 * k, 16 * k + 16)
        de.critic_step(s[sl], a[sl], y[sl])
    for k in range(n):
        de.model_actor_fit_step(s[16 * k:16 * k + 16])
    torch.cuda.synchronize()
    assert float(fe.sc.steps[0]) == float(fe.sa.steps[0]) == float(2 ** 24)
    assert torch.equal(fr.sc.steps, fe.sc.steps) and torch.equal(fr.sa.steps, fe.sa.steps)
    assert (fr.fc - fe.fc).abs().max().item() <= PARAM_ABS
    assert (fr.fa - fe.fa).abs().max().item() <= PARAM_ABS


def test_models_fit_resident_failure_falls_back(mods, monkeypatch):
    """a resident pass that loses an in-launch exchange (its timeout flag set
    after it ran) is restored and rerun on the three-launch steps, with the
    flag cleared: the same nets, moments, counts and Dropout
    call number, bit for bit, as a models_fit whose resident critic launch
    is refused outright"""
    learner, _ = mods
    from skillshot_learning_amd._capi import SkillshotError
    s, a, y = _fit_rows(16 * 40 + 5, 23)
    out = []
    for mode in ("lost_exchange", "refused"):
        d = learner.DDPG("cuda", seed=12, fused_update=True, precision="fp32")
        fu = d._fused
        real = fu.fit_critic

        def lost(*args, **kw):
            n = real(*args, **kw)
            fu.fit_timeout[0] = 1
            return n

        def refused(*args, **kw):
            raise SkillshotError("refused")

        monkeypatch.setattr(fu, "fit_critic", lost if mode == "lost_exchange" else refused)
        with pytest.warns(UserWarning, match="three-launch"):
            d.models_fit(s, a, y)
        torch.cuda.synchronize()
        assert int(fu.fit_timeout[0]) == 0 if mode == "lost_exchange" else True
        out.append((fu.fc.clone(), fu.sc.m.clone(), fu.sc.v.clone(), fu.sc.steps.clone(), fu.fa.clone(),
                    fu.sa.steps.clone(), int(d.drop_calls)))
    for x, z in zip(*out):
        assert (x == z) if isinstance(x, int) else torch.equal(x, z)
