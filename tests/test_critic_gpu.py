"""A16 on the GPU: the fused MFMA critic forward and the DDPG bootstrap target
kernel against plain PyTorch fp32 references of the same ops."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

# Kernel arithmetic: layers 1-2 with bf16 operands (inputs, W1, layer-1
# activations, W2's first 256 columns) and fp32 accumulation; W2's action
# columns and layer 3 in fp32.  EMU_* against a torch emulation of exactly
# that (fp64 accumulation), FP32_* against the plain fp32 critic.
EMU_MEAN, EMU_MAX = 5e-4, 3e-2
FP32_MEAN, FP32_MAX = 1e-2, 1.5e-1


def _bf(t):
    return t.to(torch.bfloat16).to(torch.float64)


def _emulated_q(c, s, a):
    W1, b1 = c.l1.weight.detach().double(), c.l1.bias.detach().double()
    W2, b2 = c.l2.weight.detach().double(), c.l2.bias.detach().double()
    W3, b3 = c.l3.weight.detach().double(), c.l3.bias.detach().double()
    h1 = torch.relu(_bf(s.double()) @ _bf(W1).t() + b1).float().double()
    h2 = torch.relu(_bf(h1) @ _bf(W2[:, :256]).t() + a.double() @ W2[:, 256:].float().double().t() + b2)
    h2 = h2.float().double()
    return (h2 @ W3.float().double().t() + b3).squeeze(-1).float()


@pytest.fixture(scope="module")
def mods():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from skillshot_learning_amd import learner
    from skillshot_learning_amd.critic_kernel import CriticKernel, TargetQKernel
    return learner, CriticKernel, TargetQKernel


def _nets(learner, seed=0, scale=2.0):
    torch.manual_seed(seed)
    a, c = learner.Actor().cuda(), learner.Critic().cuda()
    with torch.no_grad():
        for l in (a.l1, a.l2, a.l3, c.l1, c.l2, c.l3):
            l.weight.mul_(scale)
            l.bias.normal_(0, 0.1)
    c.eval()
    return a, c


def _obs(rows):
    return torch.rand(rows, 12, device="cuda") * torch.tensor([1, 1, 1, 1, 9.8, 1, 1, 1, 1, 9.8, 1, 1.0],
                                                             device="cuda")


@pytest.mark.parametrize("rows", [1, 31, 4096 + 17, 65536])
def test_critic_kernel_matches_torch(mods, rows):
    learner, CriticKernel, _ = mods
    a, c = _nets(learner, seed=1)
    k = CriticKernel(c)
    s = _obs(rows)
    act = torch.rand(rows, 2, device="cuda") * 2 - 1
    got = k(s, act)
    emu = (got - _emulated_q(c, s, act)).abs()
    assert emu.mean().item() < EMU_MEAN and emu.max().item() < EMU_MAX, (emu.mean().item(), emu.max().item())
    with torch.no_grad():
        ref = c(s, act).squeeze(-1)
    err = (got - ref).abs()
    assert err.mean().item() < FP32_MEAN and err.max().item() < FP32_MAX, (err.mean().item(), err.max().item())
    if rows > 1:
        assert ref.std().item() > 0.05  # non-trivial Q values


@pytest.mark.parametrize("rows", [1, 257, 8192, 40000])
def test_target_q_is_actor_then_critic(mods, rows):
    """sk_target_q: its actions equal the actor kernel's (deterministic,
    tile-per-wave launch) bit for bit, and its Q equals the critic kernel's on
    those actions bit for bit."""
    learner, CriticKernel, TargetQKernel = mods
    a, c = _nets(learner, seed=2)
    t = TargetQKernel(a, c)
    L = t.L
    L.skdiag_actor_set_mode.argtypes = [ctypes.c_int]
    s = _obs(rows)
    acts = torch.full((rows, 2), float("nan"), device="cuda")
    q = t(s, actions_out=acts)
    try:
        assert L.skdiag_actor_set_mode(1) == 0
        ref_a = t.actor_k(s)
    finally:
        L.skdiag_actor_set_mode(0)
    assert torch.equal(acts, ref_a)
    assert torch.equal(q, t.critic_k(s, acts))
    with torch.no_grad():
        ref = c(s, a(s)).squeeze(-1)
    assert (q - ref).abs().mean().item() < FP32_MEAN


def test_critic_refresh_tracks_weights(mods):
    learner, CriticKernel, _ = mods
    _, c = _nets(learner, seed=3)
    k = CriticKernel(c)
    s, act = _obs(512), torch.rand(512, 2, device="cuda") * 2 - 1
    with torch.no_grad():
        c.l3.bias.add_(1.0)
    k.refresh()
    emu = (k(s, act) - _emulated_q(c, s, act)).abs()
    assert emu.max().item() < EMU_MAX


@pytest.mark.parametrize("fused_update", [False, True])
def test_ddpg_target_uses_fused_kernel(mods, fused_update):
    """DDPG.target_q on the GPU (sk_target_q on the packed target nets, kept in
    step by soft_update, or repacked on demand after MFMA-update steps that
    moved the targets inside their Adam launches) against the torch target
    nets."""
    learner, _, _ = mods
    d = learner.DDPG("cuda", seed=4, gamma=0.9, tau=0.05, replay_capacity=4096, fused_update=fused_update, precision="bf16")
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(4):
        d.replay.add(torch.rand(512, 12, device="cuda", generator=g), torch.rand(512, 2, device="cuda") * 2 - 1,
                     torch.randn(512, device="cuda", generator=g), torch.rand(512, 12, device="cuda", generator=g),
                     torch.zeros(512, device="cuda"))
    for _ in range(3):
        d.replay_update(256)  # autograd path: creates the kernel, soft-updates and repacks
    assert (d._tq is None) == fused_update  # the MFMA update computes its target in the critic launch
    s2 = _obs(2048)
    got = d.target_q(s2)
    d.target_critic.eval()
    with torch.no_grad():
        ref = d.target_critic(s2, d.target_actor(s2)).squeeze(-1)
    err = (got - ref).abs()
    assert err.mean().item() < 2e-3 and err.max().item() < 2e-2, (err.mean().item(), err.max().item())
