"""Learner (SurveY §8 A13/A16, F1/F2) on CPU: topology/init, the reference
update rule, parameter noise by local reparameterisation, and the multi-rank
collectives (gloo, world size 2).

Parity note: TensorFlow/Keras is absent, so the update rule is restated from
SkillshotLearner.py:70-121, 386-443 and checked against its own definition
(autograd identities); it is "parity unpinned" against Keras numerics."""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from skillshot_learning_amd.learner import DDPG, Actor, Critic, ReplayRing


def test_topology_and_init():
    torch.manual_seed(0)
    a, c = Actor(), Critic()
    assert [tuple(l.weight.shape) for l in (a.l1, a.l2, a.l3)] == [(256, 12), (128, 256), (2, 128)]
    assert [tuple(l.weight.shape) for l in (c.l1, c.l2, c.l3)] == [(256, 12), (128, 258), (1, 128)]
    assert sum(p.numel() for p in a.parameters()) == 36482
    assert sum(p.numel() for p in c.parameters()) == 36609
    w = a.l2.weight.detach()  # RandomNormal(0, 0.05), SkillshotLearner.py:74
    assert abs(float(w.mean())) < 2e-3 and abs(float(w.std()) - 0.05) < 2e-3
    assert all(float(l.bias.abs().max()) == 0 for l in (a.l1, a.l2, a.l3, c.l1, c.l2, c.l3))
    lim = math.sqrt(6 / (258 + 128))  # glorot_uniform
    assert float(c.l2.weight.abs().max()) <= lim and float(c.l2.weight.abs().max()) > 0.9 * lim
    assert isinstance(c.drop, torch.nn.Dropout) and c.drop.p == 0.2


def test_actor_step_is_minus_sum_q():
    """model_actor_fit_step (:386-417): grads = -d/dtheta sum_b Q(s, mu(s)),
    critic in inference mode (no dropout), critic weights untouched."""
    d = DDPG("cpu", seed=1)
    s = torch.randn(16, 12)
    crit_before = [p.detach().clone() for p in d.model_critic.parameters()]
    d.model_critic.eval()
    ref = Actor()
    ref.load_state_dict(d.model_actor.state_dict())
    q = d.model_critic(s, ref(s)).sum()
    grads = torch.autograd.grad(-q, list(ref.parameters()))
    d.model_actor_fit_step(s)
    # first Keras Adam step: m = 0.1 g, v = 0.001 g^2, alpha = lr sqrt(0.001) / 0.1,
    # so |delta| = lr |g| / (|g| + eps / sqrt(0.001)) (epsilon-hat, not torch's)
    for (name, p), g in zip(d.model_actor.named_parameters(), grads):
        delta = p.detach() - ref.state_dict()[name]
        nz = g.abs() > 1e-6
        assert torch.all(torch.sign(delta[nz]) == -torch.sign(g[nz]))
        want = 1e-3 * g[nz].abs() / (g[nz].abs() + 1e-7 / math.sqrt(1e-3))
        assert torch.allclose(delta[nz].abs(), want, rtol=2e-3, atol=1e-9)
    for p, b in zip(d.model_critic.parameters(), crit_before):
        assert torch.equal(p.detach(), b)
    assert d.optimiser.defaults["eps"] == 1e-7 and d.optimiser.defaults["lr"] == 1e-3


def test_critic_step_mse_immediate_reward_with_dropout():
    d = DDPG("cpu", seed=2)
    s, a, r = torch.randn(16, 12), torch.rand(16, 2) * 2 - 1, torch.randn(16)
    torch.manual_seed(5)
    loss = d.critic_step(s, a, r)
    assert d.model_critic.training  # Dropout active in critic.fit (:434)
    assert torch.isfinite(loss)


def test_models_fit_one_pass_batch16():
    d = DDPG("cpu", seed=3, batch_size=16)
    n = 16 * 5 + 3
    s, a, r = torch.randn(n, 12), torch.rand(n, 2) * 2 - 1, torch.randn(n)
    d.models_fit(s, a, r)
    steps_c = d.critic_optimiser.state[next(d.model_critic.parameters())]["step"]
    steps_a = d.optimiser.state[next(d.model_actor.parameters())]["step"]
    assert int(steps_c) == 6 and int(steps_a) == 6  # ceil(83 / 16)


def test_param_noise_local_reparam_matches_explicit_weight_noise():
    """model_act_param_noise (:245-281): w' = w + w*N(0, 0.5) for every weight
    and bias.  Local reparameterisation must give the same output distribution
    as drawing explicit noisy weights per sample."""
    torch.manual_seed(0)
    a = Actor()
    with torch.no_grad():
        for l in (a.l1, a.l2, a.l3):
            l.weight.mul_(4.0)
            l.bias.normal_(0, 0.1)
    x = torch.rand(1, 12)
    n = 20000
    g = torch.Generator().manual_seed(1)
    lr = a.forward_param_noise(x.expand(n, 12), 0.5, generator=g)
    outs = []
    for _ in range(n // 500):
        ws = []
        for l in (a.l1, a.l2, a.l3):
            W = l.weight.unsqueeze(0) * (1 + 0.5 * torch.randn((500,) + tuple(l.weight.shape), generator=g))
            b = l.bias.unsqueeze(0) * (1 + 0.5 * torch.randn((500,) + tuple(l.bias.shape), generator=g))
            ws.append((W, b))
        h = x.expand(500, 12)
        for k, (W, b) in enumerate(ws):
            h = torch.einsum("bo i,bi->bo".replace(" ", ""), W, h) + b
            h = torch.tanh(h) if k == 2 else torch.relu(h)
        outs.append(h)
    ex = torch.cat(outs)
    for j in range(2):
        m1, m2 = float(lr[:, j].mean()), float(ex[:, j].mean())
        s1, s2 = float(lr[:, j].std()), float(ex[:, j].std())
        assert abs(m1 - m2) < 4 * max(s1, s2) / math.sqrt(n) * 1.5 + 1e-3
        assert abs(s1 - s2) / max(s1, s2) < 0.05
        # two-sample KS
        a_sorted, b_sorted = torch.sort(lr[:, j]).values, torch.sort(ex[:, j]).values
        grid = torch.linspace(float(min(a_sorted[0], b_sorted[0])), float(max(a_sorted[-1], b_sorted[-1])), 400)
        fa = torch.searchsorted(a_sorted, grid).float() / n
        fb = torch.searchsorted(b_sorted, grid).float() / n
        assert float((fa - fb).abs().max()) < 1.95 * math.sqrt(2 / n) * 1.3


def test_replay_ring_wraps():
    r = ReplayRing(10, "cpu")
    for k in range(3):
        s = torch.full((4, 12), float(k))
        r.add(s, torch.zeros(4, 2), torch.full((4,), float(k)), s, torch.zeros(4))
    assert r.size == 10 and r.head == 2
    assert sorted(r.r.tolist()) == [0.0, 0.0, 1.0, 1.0, 1.0, 1.0, 2.0, 2.0, 2.0, 2.0]
    s, a, rr, s2, d = r.sample(7)
    assert s.shape == (7, 12) and rr.shape == (7,)


def test_soft_update_and_bootstrap_target():
    d = DDPG("cpu", seed=4, gamma=0.9, tau=0.01, replay_capacity=1000)
    for _ in range(5):
        d.replay.add(torch.randn(64, 12), torch.rand(64, 2) * 2 - 1, torch.randn(64), torch.randn(64, 12),
                     (torch.rand(64) < 0.1).float())
    before = [p.detach().clone() for p in d.target_actor.parameters()]
    d.replay_update(32)
    after = list(d.target_actor.parameters())
    src = list(d.model_actor.parameters())
    for b, a, s in zip(before, after, src):
        assert torch.allclose(a.detach(), 0.99 * b + 0.01 * s.detach(), atol=1e-7)


# ----------------------------------------------------------------- gloo, 2 ranks
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d = DDPG("cpu", seed=100 + rank, replay_capacity=4096, rank_seed_offset=rank)  # different init per rank
        # broadcast made the weights identical
        flat = torch.cat([p.detach().reshape(-1) for p in d.model_actor.parameters()])
        # local data differs per rank
        g = torch.Generator().manual_seed(rank)
        d.replay.add(torch.randn(512, 12, generator=g), torch.rand(512, 2, generator=g) * 2 - 1,
                     torch.randn(512, generator=g), torch.randn(512, 12, generator=g), torch.zeros(512))
        # all-gather of a local minibatch
        s, a, r, s2, dd = d.replay.sample(8, generator=d.gen)
        gs, ga, gr, gs2, gd = d._allgather_batch(s, a, r, s2, dd)
        for _ in range(3):
            d.replay_update(16)
        after = torch.cat([p.detach().reshape(-1) for p in d.model_actor.parameters()]
                          + [p.detach().reshape(-1) for p in d.model_critic.parameters()])
        q.put((rank, flat.numpy().copy(), gs.numpy().copy(), s.numpy().copy(), after.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_two_rank_collectives_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict()
    for _ in range(world):
        rank, flat, gs, s, after = q.get(timeout=120)
        res[rank] = (flat, gs, s, after)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import numpy as np
    # rank 0's init broadcast to rank 1
    assert np.array_equal(res[0][0], res[1][0])
    # the gathered batch is rank 0's sample then rank 1's, identical on both ranks
    assert np.array_equal(res[0][1], res[1][1])
    assert np.array_equal(res[0][1][:8], res[0][2]) and np.array_equal(res[0][1][8:], res[1][2])
    # with all-reduced gradients every rank holds identical weights after updates
    assert np.array_equal(res[0][3], res[1][3])
