"""F1 on the GPU: the replay ring kernels (csrc/sk_replay.hip) and the fused
bootstrap target (sk_target_y) against the torch path of learner.ReplayRing /
DDPG.replay_update (exact: these are copies, gathers and one fp32 FMA)."""
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
    d = learner.DDPG("cuda", seed=3, gamma=0.9, tau=0.01)
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
                                     tau=0.05, replay_capacity=4096)
        tg = L.tick_graph(batch=128, ticks_per_graph=2, warmup=2)
        tg.run(10)
        torch.cuda.synchronize()
        out.append((torch.cat([p.detach().flatten() for p in L.model_actor.parameters()]),
                    torch.cat([p.detach().flatten() for p in L.model_critic.parameters()]),
                    L.replay.buf.clone(), int(L.replay.total_t)))
    (a1, c1, b1, t1), (a2, c2, b2, t2) = out
    assert t1 == t2 and torch.equal(b1, b2)
    assert torch.equal(a1, a2) and torch.equal(c1, c2)
