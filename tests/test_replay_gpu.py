"""F1 on the GPU: the replay ring kernels (csrc/sk_replay.hip) and the fused
bootstrap target (sk_target_y) against the torch path of learner.ReplayRing /
DDPG.replay_update (exact: these are copies, gathers and one fp32 FMA)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def learner():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from skillshot_learning_amd import learner
    return learner


def _tick(n, t):
    """a tick's [2N] rows whose values encode (tick, row)"""
    rows = 2 * n
    ids = torch.arange(rows, device="cuda", dtype=torch.float32) + 100000 * t
    s = ids[:, None] + torch.arange(12, device="cuda") / 16
    s2 = -s
    a = torch.stack([ids, ids + 0.5], 1)
    r = ids * 0.25
    done = (torch.arange(n, device="cuda") % 3 == 0).to(torch.uint8)
    return s.contiguous(), a.contiguous(), r.contiguous(), s2.contiguous(), done


@pytest.mark.parametrize("n,cap", [(5, 64), (300, 1000), (4096, 1 << 15)])
def test_insert_matches_torch_path_and_wraps(learner, n, cap):
    k = learner.ReplayRing(cap, "cuda", seed=1)
    ref = learner.ReplayRing(cap, "cuda", seed=1)
    ref._k = None  # the torch path
    for t in range(2 * cap // (2 * n) + 3):  # wraps at least twice
        s, a, r, s2, d = _tick(n, t)
        k.add_dev(s, a, r, s2, d)
        ref.add_dev(s, a, r, s2, d)
    torch.cuda.synchronize()
    assert int(k.total_t) == int(ref.total_t) == k.total
    assert torch.equal(k.buf, ref.buf)
    assert (k.head, k.size) == (int(k.head_t), int(k.size_t))


def test_sample_gathers_consistent_rows(learner):
    n, cap = 1000, 1 << 14
    ring = learner.ReplayRing(cap, "cuda", seed=7)
    for t in range(3):
        ring.add_dev(*_tick(n, t))
    B = 4096
    s, a, r, s2, d = ring.sample_dev(B)
    torch.cuda.synchronize()
    ids = s[:, 0]
    size = ring.size
    # every sampled row is a whole ring row (columns from the same transition)
    rows = ring.buf[:size]
    key = {float(v): i for i, v in enumerate(rows[:, 0].tolist())}
    idx = torch.tensor([key[float(v)] for v in ids.tolist()], device="cuda")
    assert torch.equal(s, ring.s[idx]) and torch.equal(a, ring.a[idx]) and torch.equal(r, ring.r[idx])
    assert torch.equal(s2, ring.s2[idx]) and torch.equal(d, ring.d[idx])
    # uniform over the filled range, fresh draws per call
    expected = size * (1 - (1 - 1 / size) ** B)  # distinct rows among B draws with replacement
    uniq = idx.unique().numel()
    assert abs(uniq - expected) < 0.05 * expected, (uniq, expected)
    mean = idx.float().mean().item() / (size - 1)
    assert abs(mean - 0.5) < 0.03, mean
    first = s.clone()  # sample_dev reuses its batch buffers
    s_again = ring.sample_dev(B)[0]
    assert not torch.equal(s_again, first)


def test_fused_target_matches_unfused(learner):
    torch.manual_seed(3)
    d = learner.DDPG("cuda", seed=3, gamma=0.9, tau=0.01, precision="bf16")
    s2 = torch.rand(777, 12, device="cuda")
    r = torch.randn(777, device="cuda")
    done = (torch.rand(777, device="cuda") < 0.3).float()
    y = d._target_kernel().target(s2, r, done, 0.9)
    ref = r + 0.9 * (1.0 - done) * d.target_q(s2)
    assert torch.allclose(y, ref, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("n,cap,B", [(5, 64, 256), (300, 1000, 4096), (4096, 1 << 15, 256), (256, 512, 1000)])
def test_insert_sample_fused_equals_insert_then_sample(learner, n, cap, B):
    """sk_replay_insert_sample (the learner tick's one ring launch) against
    sk_replay_insert then sk_replay_sample on an identical ring: the same
    ring, counters and minibatch bit for bit, through wrap-around and with
    rows of the current tick among the sampled ones (cap = 2n: every row)."""
    one = learner.ReplayRing(cap, "cuda", seed=3)
    two = learner.ReplayRing(cap, "cuda", seed=3)
    for t in range(2 * cap // (2 * n) + 3):
        rows = _tick(n, t)
        got = [x.clone() for x in one.add_sample_dev(*rows, B)]
        two.add_dev(*rows)
        want = [x.clone() for x in two.sample_dev(B)]
        torch.cuda.synchronize()
        for g, w in zip(got, want):
            assert torch.equal(g, w), t
        assert int(one.total_t) == int(two.total_t) == one.total == two.total
        assert torch.equal(one.buf, two.buf)
        assert not one._arrivals.any()  # every arrival slot back at 0


def test_tick_graph_fused_replay_equals_two_launches(learner, monkeypatch):
    """the captured learner tick with the ring's insert + minibatch in one
    launch (default) and in two (SK_FUSED_REPLAY=0): identical nets, ring and
    counters after the same ticks, bit for bit"""
    out = []
    for fused in ("1", "0"):
        monkeypatch.setenv("SK_FUSED_REPLAY", fused)
        L = learner.SkillshotLearner(n_envs=256, device="cuda", seed=5, exploration="action_noise", gamma=0.9,
                                     tau=0.05, replay_capacity=4096, precision="bf16")
        tg = L.tick_graph(batch=128, ticks_per_graph=2, warmup=2)
        tg.run(10)
        torch.cuda.synchronize()
        out.append((torch.cat([p.detach().flatten() for p in L.model_actor.parameters()]),
                    torch.cat([p.detach().flatten() for p in L.model_critic.parameters()]),
                    L.replay.buf.clone(), int(L.replay.total_t)))
    (a1, c1, b1, t1), (a2, c2, b2, t2) = out
    assert t1 == t2 and torch.equal(b1, b2)
    assert torch.equal(a1, a2) and torch.equal(c1, c2)


@pytest.mark.parametrize("n,cap", [(5, 64), (300, 1000), (4096, 1 << 14)])
def test_step_insert_equals_step_then_insert(learner, n, cap):
    """sk_env_step_insert (the env step with the ring insert in its launch)
    against sk_env_step followed by sk_replay_insert: the same step outputs,
    ring and counters bit for bit, every tick, through wrap-around and
    episode restarts (tick limit 40)"""
    from skillshot_learning_amd.vec_env import VecSkillshotGame
    envs = [VecSkillshotGame(n, device="cuda", seed=11, tick_limit=40) for _ in range(2)]
    rings = [learner.ReplayRing(cap, "cuda", seed=3) for _ in range(2)]
    obs = [e.reset(random_positions=True) or e.observe()[0].clone() for e in envs]
    gen = torch.Generator(device="cuda").manual_seed(4)
    for t in range(2 * cap // (2 * n) + 60):
        act = torch.rand((2, n, 2), device="cuda", generator=gen) * 2.4 - 1.2
        o1 = envs[0].step_insert(act, obs[0], rings[0], reset_obs=True)
        o2 = envs[1].step(act, obs=True, reward="looking", auto_reset=True, reset_obs=True)
        rings[1].add_dev(obs[1].view(-1, 12), act.view(-1, 2), o2["reward"].view(-1), o2["obs"].view(-1, 12),
                         o2["done"])
        torch.cuda.synchronize()
        for k in ("obs", "reward", "done", "winner", "obs_reset"):
            assert torch.equal(o1[k], o2[k]), (t, k)
        assert int(rings[0].total_t) == int(rings[1].total_t) == rings[0].total == rings[1].total
        assert torch.equal(rings[0].buf, rings[1].buf), t
        assert not rings[0].arrivals().any()
        obs = [o1["obs_reset"], o2["obs_reset"]]
    assert envs[0].counters() == envs[1].counters()
    assert envs[0].counters()["dones"] > 0


@pytest.mark.parametrize("precision,B,gamma", [("fp32", 256, 0.9), ("fp32", 256, 0.0), ("fp32", 100, 0.9),
                                                ("fp32", 1000, 0.9), ("bf16", 256, 0.9), ("bf16", 100, 0.0),
                                                ("bf16", 1000, 0.9)])
def test_critic_step_sampled_equals_sample_then_step(learner, precision, B, gamma):
    """the critic step drawing its minibatch from the ring inside its (first)
    launch (sk_critic_grad_f32_sampled, sk_critic_grad_bootstrap_sampled)
    against sample_dev + the critic step on those rows: identical sample
    buffers, losses and nets, bit for bit, over several steps (fp32 at 1000
    rows: the unsliced path, gather as its own launch); the reported losses to
    1e-5 (their per-workgroup sums arrive by atomics)"""
    out = []
    for sampled in (True, False):
        torch.manual_seed(0)
        d = learner.DDPG("cuda", seed=2, gamma=gamma, tau=0.05, replay_capacity=3000, precision=precision)
        g = torch.Generator(device="cuda").manual_seed(9)
        for t in range(3):
            d.replay.add_dev(torch.rand(1000, 12, device="cuda", generator=g),
                             torch.rand(1000, 2, device="cuda", generator=g),
                             torch.randn(1000, device="cuda", generator=g),
                             torch.rand(1000, 12, device="cuda", generator=g),
                             (torch.rand(1000, device="cuda", generator=g) < 0.2).float())
        losses, batches = [], []
        for _ in range(4):
            if sampled:
                lc, la = d.update_sampled(B)
            else:
                lc, la = d.replay_update(B, device_sampling=True)
            losses.append((lc.clone(), la.clone()))
            batches.append([x.clone() for x in d.replay._batch_bufs(B)])
        torch.cuda.synchronize()
        out.append((losses, batches, torch.cat([p.detach().flatten() for p in d.model_actor.parameters()]),
                    torch.cat([p.detach().flatten() for p in d.model_critic.parameters()])))
    (l1, b1, a1, c1), (l2, b2, a2, c2) = out
    for x, y in zip(b1, b2):
        for u, v in zip(x, y):
            assert torch.equal(u, v)
    for (x1, y1), (x2, y2) in zip(l1, l2):  # the loss sums arrive by float atomics: order-dependent rounding
        assert torch.allclose(x1, x2, rtol=1e-5, atol=0) and torch.allclose(y1, y2, rtol=1e-5, atol=0)
    assert torch.equal(a1, a2) and torch.equal(c1, c2)


@pytest.mark.parametrize("precision,exploration", [("fp32", "action_noise"), ("fp32", "param_noise"),
                                                   ("bf16", "action_noise")])
def test_tick_graph_replay_modes_equal(learner, monkeypatch, precision, exploration):
    """the captured learner tick with the actor forward, the env step and the
    ring insert in one launch and the minibatch drawn in the critic's
    (SK_FUSED_REPLAY=2, default; fp32), with the actor as its own launch
    (SK_FUSED_ACT=0), with the insert + minibatch as one launch (1), and as two
    (0): identical nets, ring and counters after the same ticks, bit for bit
    (32-row actor tiles everywhere: SK_FWD16=0)"""
    monkeypatch.setenv("SK_FWD16", "0")
    monkeypatch.setenv("SK_TICK_OVERLAP", "0")  # the sequential tick (the overlapped one: test_tick_overlap_*)
    out = []
    for fused, act in (("2", "1"), ("2", "0"), ("1", "1"), ("0", "1")):
        monkeypatch.setenv("SK_FUSED_REPLAY", fused)
        monkeypatch.setenv("SK_FUSED_ACT", act)
        L = learner.SkillshotLearner(n_envs=256, device="cuda", seed=5, exploration=exploration, gamma=0.9,
                                     tau=0.05, replay_capacity=4096, precision=precision, tick_limit=50)
        tg = L.tick_graph(batch=128, ticks_per_graph=2, warmup=2)
        tg.run(30)
        torch.cuda.synchronize()
        out.append((torch.cat([p.detach().flatten() for p in L.model_actor.parameters()]),
                    torch.cat([p.detach().flatten() for p in L.model_critic.parameters()]),
                    L.replay.buf.clone(), int(L.replay.total_t), L.game_environment.counters()))
    assert out[0][4]["dones"] > 0
    for a, c, b, t, k in out[1:]:
        assert t == out[0][3] and torch.equal(b, out[0][2])
        assert torch.equal(a, out[0][0]) and torch.equal(c, out[0][1])
        assert k == out[0][4]


@pytest.mark.parametrize("tile", ["32", "16"])
@pytest.mark.parametrize("n", [256, 4096, 300, 302])
@pytest.mark.parametrize("noise", ["none", "param", "action"])
def test_act_step_equals_actor_then_step_insert(learner, monkeypatch, n, noise, tile):
    """sk_env_act_step (the fp32 actor forward, the env step and the ring
    insert in one launch) against sk_actor_forward_f32 (32-row tiles) then
    sk_env_step_insert: the same actions, step outputs, ring, counters and
    noise call number bit for bit, every tick, through restarts (300 games: a
    partial last 16-game tile; 302: N % 4 != 0, the two-launch fallback).
    tile 16: k_act_step16 (8 games per workgroup, SK_ACT16=1) against the
    16-row forward (SK_FWD16=1)"""
    from skillshot_learning_amd.actor_kernel import ActorKernel32
    from skillshot_learning_amd.vec_env import VecSkillshotGame
    monkeypatch.setenv("SK_FWD16", "1" if tile == "16" else "0")
    monkeypatch.setenv("SK_ACT16", "1" if tile == "16" else "0")
    torch.manual_seed(1)
    actor = learner.Actor().cuda()
    sd, asd = {"none": (0.0, 0.0), "param": (0.5, 0.0), "action": (0.0, 0.15)}[noise]
    ks = [ActorKernel32(actor, seed=9) for _ in range(2)]
    envs = [VecSkillshotGame(n, device="cuda", seed=11, tick_limit=30) for _ in range(2)]
    rings = [learner.ReplayRing(1 << 13, "cuda", seed=3) for _ in range(2)]
    obs = [e.observe()[0].clone() for e in envs]
    for t in range(45):
        o1 = envs[0].act_step(ks[0], obs[0], noise_sd=sd, action_sd=asd, ring=rings[0])
        act = ks[1](obs[1].view(-1, 12), noise_sd=sd, action_sd=asd).view(2, n, 2)
        o2 = envs[1].step_insert(act, obs[1], rings[1], reset_obs=True)
        torch.cuda.synchronize()
        assert torch.equal(o1["actions"], act), t
        for k in ("obs", "reward", "done", "winner", "obs_reset"):
            assert torch.equal(o1[k], o2[k]), (t, k)
        assert torch.equal(rings[0].buf, rings[1].buf), t
        assert int(rings[0].total_t) == int(rings[1].total_t)
        assert torch.equal(ks[0]._ctr, ks[1]._ctr)
        obs = [o1["obs_reset"], o2["obs_reset"]]
    assert envs[0].counters() == envs[1].counters()
    assert envs[0].counters()["dones"] > 0


@pytest.mark.parametrize("precision,exploration,tile", [("fp32", "action_noise", "32"), ("fp32", "param_noise", "32"),
                                                        ("bf16", "action_noise", "32"), ("fp32", "action_noise", "16"),
                                                        ("fp32", "param_noise", "16")])
def test_tick_overlap_equals_serial(learner, monkeypatch, precision, exploration, tile):
    """the overlapped learner tick (acting launches on a second stream beside
    the update, minibatch keyed on the count before the tick's insert, the
    insert's rows excluded; joined before the actor's Adam launch): 20
    graph-replayed ticks equal the same ticks captured on one stream
    (SK_TICK_OVERLAP=serial) bit for bit -- nets, target nets, ring,
    counters -- i.e. the two streams share no data they race on; and (fp32)
    the fused form, the acting launch run by the actor gradient's backward
    launch (SK_TICK_OVERLAP=fused, sk_actor_grad_f32_step), equals them too"""
    monkeypatch.setenv("SK_ACT16", "1" if tile == "16" else "0")
    out = []
    for mode in ("1", "serial") + (("fused", "fused-actor") if precision == "fp32" else ()):
        monkeypatch.setenv("SK_FUSE_ACT_IN", "actor" if mode == "fused-actor" else "critic")
        mode = mode.split("-")[0]
        monkeypatch.setenv("SK_TICK_OVERLAP", mode)
        L = learner.SkillshotLearner(n_envs=256, device="cuda", seed=7, exploration=exploration, gamma=0.9,
                                     tau=0.05, replay_capacity=4096, precision=precision, tick_limit=50)
        tg = L.tick_graph(batch=128, ticks_per_graph=2, warmup=2)
        assert tg.overlap and (tg.side is None) == (mode != "1") and tg.fuse_act == (mode == "fused")
        tg.run(10)
        torch.cuda.synchronize()
        out.append((torch.cat([p.detach().flatten() for p in L.model_actor.parameters()]),
                    torch.cat([p.detach().flatten() for p in L.model_critic.parameters()]),
                    torch.cat([p.detach().flatten() for p in L.ddpg.target_actor.parameters()]),
                    L.replay.buf.clone(), int(L.replay.total_t), L.game_environment.counters(
                        stream=ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))))
    (a1, c1, t1, b1, n1, k1) = out[0]
    assert k1["dones"] > 0
    for a2, c2, t2, b2, n2, k2 in out[1:]:
        assert n1 == n2 and torch.equal(b1, b2)
        assert torch.equal(a1, a2) and torch.equal(c1, c2) and torch.equal(t1, t2)
        assert k1 == k2


def test_overlap_sample_excludes_rows_being_written(learner):
    """ring_row with exclude = E keys on the count before an insert and draws
    only the min(count, capacity - E) most recent rows: never a row the E-row
    insert after that count overwrites (a full ring wraps here)"""
    from skillshot_learning_amd.update_kernel import RingSample  # noqa: F401 (the ABI struct)
    cap, E, B = 1000, 300, 4096
    d = learner.DDPG("cuda", seed=1, gamma=0.0, replay_capacity=cap, precision="fp32")
    ring = d.replay
    for t in range(9):  # 2,700 rows: wrapped twice
        ids = torch.arange(E, device="cuda", dtype=torch.float32) + E * t
        ring.add_dev(ids[:, None].expand(E, 12).contiguous(), torch.zeros(E, 2, device="cuda"),
                     torch.zeros(E, device="cuda"), torch.zeros(E, 12, device="cuda"), torch.zeros(E, device="cuda"))
    count = torch.tensor(int(ring.total_t), dtype=torch.int64, device="cuda")
    d._fused.critic_step_sampled(ring, B, total=count, exclude=E)
    s = ring._batch_bufs(B)[0]
    torch.cuda.synchronize()
    got = s[:, 0].long()
    total = int(count)
    lo = total - min(total, cap - E)  # the oldest row id still eligible
    assert int(got.min()) >= lo and int(got.max()) < total
    assert got.unique().numel() > 0.9 * (cap - E)  # uniform over the eligible rows
    # the overlapped draw's window is exactly the sequential
    # (reference-order) tick's window minus the E rows that tick inserts.
    # The sequential tick draws after its insert, keyed on count + E with no
    # exclusion: rows [count + E - min(count + E, cap), count + E)
    ids = torch.arange(E, device="cuda", dtype=torch.float32) + total
    ring.add_dev(ids[:, None].expand(E, 12).contiguous(), torch.zeros(E, 2, device="cuda"),
                 torch.zeros(E, device="cuda"), torch.zeros(E, 12, device="cuda"), torch.zeros(E, device="cuda"))
    d._fused.critic_step_sampled(ring, B, exclude=0)
    seq = ring._batch_bufs(B)[0][:, 0].long()
    torch.cuda.synchronize()
    after = int(ring.total_t)
    assert after == total + E
    seq_window = set(range(after - min(after, cap), after))
    assert set(seq.tolist()) <= seq_window
    over_window = set(range(lo, total))
    assert over_window == seq_window - set(range(total, total + E))
    assert set(got.tolist()) <= over_window


@pytest.mark.parametrize("batch", [128, 1024])  # sliced schedule (one shared launch) / not (two launches)
@pytest.mark.parametrize("noise", ["param", "action"])
@pytest.mark.parametrize("carrier,tile", [("actor", "32"), ("critic", "32"), ("critic", "16")])
def test_grad_step_job_equals_separate_launches(learner, monkeypatch, batch, noise, carrier, tile):
    """sk_env_act_step_job + sk_actor_grad_f32_step / sk_critic_grad_f32_sampled_step
    (the acting tick run in a gradient step's backward launch) against the
    gradient step and sk_env_act_step as separate launches: the net after
    each Adam step, the actions, the env outputs, the ring and the noise call
    number, bit for bit, every tick"""
    from skillshot_learning_amd import _capi
    from skillshot_learning_amd.actor_kernel import ActorKernel32
    from skillshot_learning_amd.vec_env import VecSkillshotGame
    monkeypatch.setenv("SK_FWD16", "0")
    monkeypatch.setenv("SK_ACT16", "1" if tile == "16" else "0")
    n = 256
    sd, asd = {"param": (0.5, 0.0), "action": (0.0, 0.15)}[noise]
    out = []
    for fused in (True, False):
        d = learner.DDPG("cuda", seed=1, gamma=0.9, tau=0.05, replay_capacity=4096, precision="fp32")
        fu = d._fused
        assert fu.sliced(batch) == (batch <= 512)
        k = ActorKernel32(d.model_actor, seed=9)
        env = VecSkillshotGame(n, device="cuda", seed=11, tick_limit=30)
        ring = learner.ReplayRing(1 << 13, "cuda", seed=3)
        obs = env.observe()[0].clone()
        g = torch.Generator(device="cuda").manual_seed(5)
        job = _capi.SkStepJob()
        rec = []
        for t in range(6):
            s = torch.rand((batch, 12), device="cuda", generator=g) * 2 - 1
            if carrier == "actor":
                if fused:
                    o = env.act_step(k, obs, noise_sd=sd, action_sd=asd, ring=ring, job=job)
                    fu.actor_step(s, step_job=job)
                else:
                    o = env.act_step(k, obs, noise_sd=sd, action_sd=asd, ring=ring)
                    fu.actor_step(s)
            elif t == 0:  # the critic draws from the ring: fill it first
                o = env.act_step(k, obs, noise_sd=sd, action_sd=asd, ring=ring)
            elif fused:
                o = env.act_step(k, obs, noise_sd=sd, action_sd=asd, ring=ring, job=job)
                fu.critic_step_sampled(ring, batch, gamma=0.9, exclude=2 * n, step_job=job)
            else:
                fu.critic_step_sampled(ring, batch, gamma=0.9, exclude=2 * n)
                o = env.act_step(k, obs, noise_sd=sd, action_sd=asd, ring=ring)
            torch.cuda.synchronize()
            rec.append((fu.fa.clone(), fu.fc.clone(), o["actions"].clone(), o["obs"].clone(), o["reward"].clone(),
                        o["done"].clone(), ring.buf.clone(), k._ctr.clone()))
            obs = o["obs_reset"]
        out.append((rec, env.counters()))
    (r1, c1), (r2, c2) = out
    for t, (x, y) in enumerate(zip(r1, r2)):
        for i, (u, v) in enumerate(zip(x, y)):
            assert torch.equal(u, v), (t, i)
    assert c1 == c2


@pytest.mark.parametrize("exclude", [0, 300])
def test_sampled_rows_equal_restated_ring_row(learner, exclude):
    """the rows the critic launch gathers (ring_row, csrc/sk_mlp.hpp) against
    a restatement on the host: Philox4x32-10 of (b, draw, count lo, count hi)
    under the ring's seed (rng.philox4x32_10), u53 = (x << 32 | y) >> 11,
    index = (u53 * size) >> 53, or with an exclusion E: the
    min(count, cap - E) newest rows, (count - el + k) mod cap.  Row ids, bit
    for bit, on a ring that wrapped twice"""
    from skillshot_learning_amd.rng import philox4x32_10
    cap, E, B = 1000, 300, 512
    d = learner.DDPG("cuda", seed=1, gamma=0.0, replay_capacity=cap, precision="fp32")
    ring = d.replay
    for t in range(9):
        ids = torch.arange(E, device="cuda", dtype=torch.float32) + E * t
        ring.add_dev(ids[:, None].expand(E, 12).contiguous(), torch.zeros(E, 2, device="cuda"),
                     torch.zeros(E, device="cuda"), torch.zeros(E, 12, device="cuda"), torch.zeros(E, device="cuda"))
    count = int(ring.total_t)
    draw = ring._draws
    d._fused.critic_step_sampled(ring, B, total=torch.tensor(count, dtype=torch.int64, device="cuda"),
                                 exclude=exclude)
    got = ring._batch_bufs(B)[0][:, 0].long().cpu()
    b = torch.arange(B, dtype=torch.int64)
    x, y, _, _ = philox4x32_10(b, draw, count & 0xFFFFFFFF, count >> 32, ring.seed & 0xFFFFFFFF, ring.seed >> 32)
    want = []
    for xi, yi in zip(x.tolist(), y.tolist()):
        u53 = ((xi << 32) | yi) >> 11
        if exclude <= 0:
            idx = (u53 * min(count, cap)) >> 53
        else:
            el = min(count, cap - exclude)
            idx = (count - el + ((u53 * el) >> 53)) % cap
        want.append(idx + cap * ((count - 1 - idx) // cap))  # the id the ring row holds (latest write)
    assert got.tolist() == want


@pytest.mark.parametrize("overlap", [None, "fused"])
def test_tick_graph_odd_ticks_per_graph(learner, overlap):
    """ticks_per_graph need not be even: an odd count is
    two graphs replayed alternately.  Six ticks as 3 + 3 (two run() calls,
    the second starting in the other phase), as 1 x 6 and as 2 x 3 end in the
    same nets, ring, game state and next observation, bit for bit"""
    out = []
    for tpg, runs in ((3, (1, 1)), (1, (6,)), (2, (3,))):
        L = learner.SkillshotLearner(n_envs=256, device="cuda", seed=7, exploration="action_noise", gamma=0.9,
                                     tau=0.05, replay_capacity=4096, precision="fp32")
        tg = L.tick_graph(batch=128, ticks_per_graph=tpg, warmup=2, overlap=overlap)
        for r in runs:
            tg.run(r)
        torch.cuda.synchronize()
        st = L.game_environment.state_dict()
        out.append((torch.cat([p.detach().flatten() for p in L.model_actor.parameters()]),
                    torch.cat([p.detach().flatten() for p in L.model_critic.parameters()]),
                    L.replay.buf.clone(), int(L.replay.total_t), tg.obs.clone(),
                    {k: v for k, v in st.items() if k != "step_counter"}, tg.mode))
    a0, c0, b0, t0, o0, s0, m0 = out[0]
    for a, c, b, t, o, s, m in out[1:]:
        assert m == m0
        assert t == t0 and torch.equal(b, b0)
        assert torch.equal(a, a0) and torch.equal(c, c0)
        assert torch.equal(o, o0)
        for k in s0:
            assert (s[k] == s0[k]).all(), k
