"""A13/F2 on the GPU: the fused MFMA actor kernel against a plain PyTorch fp32
reference of the same op, and the learner loop end to end."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

# The kernel's op: layers 1-2 on MFMA with bf16 operands (inputs, weights,
# layer-1 activations), fp32 accumulation and epilogues; layer 3 on the fp32
# VALU (fp32 layer-2 activations and W3).  Against a torch reference of exactly
# that op (same roundings, fp64 accumulation) only accumulation order differs,
# but that can move a hidden activation across a bf16 rounding boundary (one
# bf16 ulp, 2^-8 relative), so the bar is a mean and a max: EMU_*.  Against the
# pure fp32 actor the operand rounding itself shows: FP32_* at 4x the
# reference init scale (pre-activations ~O(10)).
EMU_MEAN, EMU_MAX = 5e-4, 3e-2
FP32_MEAN, FP32_MAX = 5e-3, 8e-2


def _bf(t):
    return t.to(torch.bfloat16).to(torch.float64)


def _emulated(a, x):
    """The kernel's arithmetic in torch: bf16 operands for layers 1-2, fp32
    for layer 3, fp64 accumulation."""
    h = x.double()
    for k, l in enumerate((a.l1, a.l2, a.l3)):
        rnd = _bf if k < 2 else (lambda t: t.float().double())
        h = rnd(h) @ rnd(l.weight.detach()).t() + l.bias.detach().double()
        h = torch.tanh(h) if k == 2 else torch.relu(h).float().double()
    return h.float()


@pytest.fixture(scope="module")
def mods():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from skillshot_learning_amd import learner
    from skillshot_learning_amd.actor_kernel import ActorKernel
    return learner, ActorKernel


def _actor(learner, scale=4.0, seed=0):
    torch.manual_seed(seed)
    a = learner.Actor().cuda()
    with torch.no_grad():
        for l in (a.l1, a.l2, a.l3):
            l.weight.mul_(scale)
            l.bias.normal_(0, 0.1)
    return a


@pytest.mark.parametrize("rows", [1, 31, 32, 4096 + 17, 131072])
def test_actor_kernel_matches_torch_fp32(mods, rows):
    learner, ActorKernel = mods
    a = _actor(learner)
    k = ActorKernel(a)
    x = torch.rand(rows, 12, device="cuda") * torch.tensor([1, 1, 1, 1, 9.8, 1, 1, 1, 1, 9.8, 1, 1.0],
                                                          device="cuda")
    got = k(x)
    emu = (got - _emulated(a, x)).abs()
    assert emu.mean().item() < EMU_MEAN and emu.max().item() < EMU_MAX, (emu.mean().item(), emu.max().item())
    err = (got - a(x)).abs()
    assert err.mean().item() < FP32_MEAN and err.max().item() < FP32_MAX, (err.mean().item(), err.max().item())
    assert got.abs().max().item() > 0.2  # non-trivial outputs


def test_actor_kernel_refresh_tracks_weights(mods):
    learner, ActorKernel = mods
    a = _actor(learner, seed=3)
    k = ActorKernel(a)
    x = torch.rand(256, 12, device="cuda")
    with torch.no_grad():
        a.l3.bias.add_(0.5)
    k.refresh()
    emu = (k(x) - _emulated(a, x)).abs()
    assert emu.mean().item() < EMU_MEAN and emu.max().item() < EMU_MAX


def test_param_noise_kernel_distribution(mods):
    """Per-row parameter noise: moments match the torch local-reparameterisation
    reference (itself checked against explicit weight noise on CPU)."""
    learner, ActorKernel = mods
    a = _actor(learner, seed=5)
    k = ActorKernel(a, seed=11)
    n = 200000
    x = torch.rand(1, 12, device="cuda").expand(n, 12).contiguous()
    got = k(x, noise_sd=0.5)
    g = torch.Generator(device="cuda").manual_seed(2)
    want = a.forward_param_noise(x, 0.5, generator=g)
    for j in range(2):
        m1, m2 = got[:, j].mean().item(), want[:, j].mean().item()
        s1, s2 = got[:, j].std().item(), want[:, j].std().item()
        # MC error ~ s/sqrt(n) = 0.002; bf16 operands of the mean and variance
        # chains add a small deterministic bias
        assert abs(m1 - m2) < 0.01 + 5 * max(s1, s2) / math.sqrt(n), (j, m1, m2)
        assert abs(s1 - s2) / max(s1, s2) < 0.02, (j, s1, s2)
    # fresh noise per call and per row
    again = k(x, noise_sd=0.5)
    assert (again - got).abs().mean().item() > 1e-3
    assert got[:, 0].unique().numel() > n // 2


def _ctr_is(k, call):
    """the call number is `call` and every arrival slot (word 1 and the 8
    group lines, SK_ACTOR_COUNTER_WORDS) is back at 0"""
    c = k._ctr.tolist()
    return c[0] == call and not any(c[1:])


@pytest.mark.parametrize("rows", [8192, 131072])  # tile-per-workgroup and tile-per-wave launch modes
def test_noise_counter_advances_in_kernel(mods, rows):
    """sk_actor_forward_advance: noisy call k draws with call number k (the
    same noise as an explicit sk_actor_forward(call=k)), the counter holds k
    afterwards with the arrival slot back at 0, deterministic calls leave it."""
    import ctypes
    learner, ActorKernel = mods
    a = _actor(learner, seed=7)
    k = ActorKernel(a, seed=13)
    x = torch.rand(rows, 12, device="cuda")
    ref = torch.empty(rows, 2, device="cuda")
    for call in (1, 2, 3):
        got = k(x, noise_sd=0.5)
        rc = k.L.sk_actor_forward(ctypes.c_void_p(k.buf.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                  ctypes.c_void_p(ref.data_ptr()), rows, 0.5, k.seed, call, k._stream())
        assert rc == 0
        assert torch.equal(got, ref), call
        assert _ctr_is(k, call), call
    k(x)
    assert _ctr_is(k, 3)


@pytest.mark.parametrize("rows", [8192, 65536])  # tile-per-workgroup and tile-per-wave launch modes
def test_action_noise_in_kernel(mods, rows):
    """model_act_action_noise (:229-243) in the bf16 kernel
    (sk_actor_forward_noise): the clean tanh outputs + N(0, 0.15) per output,
    unclipped; the call counter advances per launch, so repeated calls and
    graph replays draw fresh noise; parameter noise alongside still works."""
    learner, ActorKernel = mods
    a = _actor(learner, seed=9)
    k = ActorKernel(a, seed=5)
    x = torch.rand(rows, 12, device="cuda")
    clean = k(x)
    a1 = k(x, action_sd=0.15)
    a2 = k(x, action_sd=0.15)
    torch.cuda.synchronize()
    assert _ctr_is(k, 2)
    z = ((a1 - clean) / 0.15).double().cpu().flatten()
    assert abs(float(z.mean())) < 0.03 and abs(float(z.std()) - 1.0) < 0.03
    assert abs(float((z.abs() < 1).double().mean()) - 0.6827) < 0.02  # normal, not uniform
    assert float(a1.abs().max()) > 1.0  # unclipped, as the reference adds after tanh
    assert not torch.equal(a1, a2)
    both = k(x, noise_sd=0.5, action_sd=0.15)
    assert _ctr_is(k, 3) and bool(torch.isfinite(both).all())


def test_learner_replay_training_runs(mods):
    learner, _ = mods
    L = learner.SkillshotLearner(n_envs=2048, seed=1, tick_limit=300, replay_capacity=1 << 16, gamma=0.9, tau=0.005, precision="bf16")
    # games start their first episode in the learner's start mode (random)
    pos = L.game_environment.state_dict()["pos"]
    assert torch.unique(torch.as_tensor(pos), dim=0).shape[0] > 1900
    stats = L.train_ticks(40, batch=512)
    assert len(stats) > 0
    assert all(torch.isfinite(c) and torch.isfinite(a) for c, a in stats)
    assert L.replay.size == min(1 << 16, 40 * 2 * 2048)
    c = L.game_environment.counters()
    assert c["dones"] > 0 and c["hits_p1"] + c["hits_p2"] == c["dones"]  # hits end episodes (no tick cap yet)


def test_learner_reference_epochs(mods):
    """model_train with the reference update rule (batch 16, one pass) on a few
    games with a short tick limit (SkillshotLearner.main uses 200, :688)."""
    learner, _ = mods
    L = learner.SkillshotLearner(n_envs=4, seed=2, tick_limit=60, exploration="param_noise", precision="bf16")
    before = [p.detach().clone() for p in L.model_actor.parameters()]
    prog = L.model_train(epochs=2)
    assert len(prog["epoch_ticks"]) == 2
    assert all(int(t.max()) <= 60 for t in prog["epoch_ticks"])
    moved = sum(float((p.detach() - b).abs().sum()) for p, b in zip(L.model_actor.parameters(), before))
    assert moved > 0
    for mode in ("action_noise", None):
        L.exploration = mode or "deterministic"
        act = L.model_act(L.prepare_states())
        assert act.shape == (2, 4, 2) and torch.isfinite(act).all()


def test_model_train_saves_progress_boards_models(mods, tmp_path):
    """model_train(save_progress, save_boards) (:370-384): the models, one
    progress row per (epoch, game) and game 0's board after every tick it was
    live, each board the rasterised engine state; models load back."""
    import numpy as np
    from skillshot_learning_amd.game import rasterize_board
    learner, _ = mods
    L = learner.SkillshotLearner(n_envs=1, seed=4, tick_limit=40, precision="bf16")  # one game, as the reference plays
    L.save_location = str(tmp_path / "training_models")
    prog = L.model_train(epochs=2, save_progress=True, save_boards=True)
    df = L.load_training_progress()
    assert df.shape[0] == 2
    assert df["epoch_ticks"].tolist() == [int(x) for t in prog["epoch_ticks"] for x in t]
    boards = L.load_training_boards()
    assert len(boards) == 2
    for e in range(2):
        assert boards[e].shape == (int(prog["epoch_ticks"][e][0]), 250, 250)
    st = L.game_environment.state_dict()  # the final board of epoch 1 is the game's state now
    pos, qpos, rot = st["pos"][0], st["qpos"][0], st["rot"][0]
    flags = int(np.uint32(st["misc"][0, 1]))
    want = rasterize_board(np.zeros((250, 250), dtype=np.int64), [pos[:2], pos[2:]], rot, [qpos[:2], qpos[2:]],
                           [flags & 0xFF, (flags >> 8) & 0xFF])
    assert np.array_equal(boards[1][-1], want)
    w = [p.detach().clone() for p in L.model_actor.parameters()]
    with torch.no_grad():
        for p in L.model_actor.parameters():
            p.add_(1.0)
    assert L.load_actor_critic_models()
    assert all(torch.equal(p, q) for p, q in zip(L.model_actor.parameters(), w))


def test_learner_reference_epochs_full_reward(mods):
    """model_train with the alternative reward functions (:324-326)."""
    learner, _ = mods
    for reward in ("full", "simple"):
        L = learner.SkillshotLearner(n_envs=8, seed=4, tick_limit=80, exploration="param_noise", precision="bf16")
        before = [p.detach().clone() for p in L.model_critic.parameters()]
        prog = L.model_train(epochs=1, reward=reward)
        assert len(prog["epoch_ticks"]) == 1
        moved = sum(float((p.detach() - b).abs().sum()) for p, b in zip(L.model_critic.parameters(), before))
        assert moved > 0


def test_tick_graph_replays_train(mods):
    """The replay-rule tick captured as one hipGraph: replays keep inserting
    at the device-side head, draw fresh parameter noise and keep training."""
    learner, _ = mods
    L = learner.SkillshotLearner(n_envs=1024, seed=6, tick_limit=300, replay_capacity=1 << 14, gamma=0.9, tau=0.01, precision="bf16")
    tg = L.tick_graph(batch=256, updates_per_tick=1, ticks_per_graph=2)
    size0 = int(L.replay.size_t)
    head0 = int(L.replay.head_t)
    a0 = tg.act.clone()
    w0 = [p.detach().clone() for p in L.model_actor.parameters()]
    t0 = [p.detach().clone() for p in L.ddpg.target_actor.parameters()]
    ctr0 = int(L.actor_kernel.counter)
    step0 = L.game_environment.step_counter
    tg.run(5)
    torch.cuda.synchronize()
    rows = 5 * 2 * 2 * 1024
    assert int(L.replay.size_t) == min(1 << 14, size0 + rows)
    assert int(L.replay.head_t) == (head0 + rows) % (1 << 14)
    assert (L.replay.size, L.replay.head) == (int(L.replay.size_t), int(L.replay.head_t))
    assert int(L.actor_kernel.counter) == ctr0 + 10            # one noisy call per tick
    assert L.game_environment.step_counter == step0 + 10       # device step counter advanced per tick
    assert (tg.act - a0).abs().mean().item() > 1e-3             # fresh actions
    assert sum(float((p.detach() - w).abs().sum()) for p, w in zip(L.model_actor.parameters(), w0)) > 0
    assert sum(float((p.detach() - w).abs().sum()) for p, w in zip(L.ddpg.target_actor.parameters(), t0)) > 0
    for p in list(L.model_actor.parameters()) + list(L.model_critic.parameters()):
        assert torch.isfinite(p).all()
    # the ring holds the graph's transitions: finite obs, actions in [-1, 1]
    assert torch.isfinite(L.replay.s[:L.replay.size]).all()
    assert L.replay.a[:L.replay.size].abs().max().item() <= 1.0


@pytest.mark.parametrize("rows", [1, 33, 4113, 8192, 40000])
def test_actor_launch_modes_agree(mods, rows):
    """Tile-per-wave and tile-per-workgroup launches draw the same noise
    (same Philox counters) and differ only in layer 3's fp32 summation order."""
    import ctypes
    learner, ActorKernel = mods
    a = _actor(learner, seed=7)
    k = ActorKernel(a, seed=3)
    L = k.L
    L.skdiag_actor_set_mode.argtypes = [ctypes.c_int]
    L.skdiag_actor_set_mode.restype = ctypes.c_int
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    x = torch.rand(rows, 12, device="cuda")
    try:
        for sd in (0.0, 0.5):
            outs = []
            for mode in (1, 2):
                assert L.skdiag_actor_set_mode(mode) == 0
                y = torch.full((rows, 2), float("nan"), device="cuda")
                assert L.sk_actor_forward(p(k.buf), p(x), p(y), rows, sd, 99, 5, stream) == 0
                outs.append(y)
            torch.cuda.synchronize()
            assert torch.isfinite(outs[0]).all() and torch.isfinite(outs[1]).all()
            assert (outs[0] - outs[1]).abs().max().item() < 1e-5, (sd, rows)
    finally:
        L.skdiag_actor_set_mode(0)
