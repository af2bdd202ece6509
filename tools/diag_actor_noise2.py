import sys, torch, math
sys.path.insert(0, "/root/repo")
from skillshot_learning_amd import learner
from skillshot_learning_amd.actor_kernel import ActorKernel
torch.manual_seed(5)
a = learner.Actor().cuda()
n = 400000
x = torch.rand(1, 12, device="cuda").expand(n, 12).contiguous()
with torch.no_grad():
    a.l3.weight.zero_(); a.l3.bias.copy_(torch.tensor([1.0, -0.5]))
k = ActorKernel(a, seed=3)
for sd in (0.1, 0.5):
    y = torch.atanh(k(x, noise_sd=sd).clamp(-0.999999, 0.999999).double())
    print(f"T1 W3=0 sd={sd}: pre-act mean {y.mean(0).tolist()} std {y.std(0).tolist()} expected std {[sd*1.0, sd*0.5]}")
# T2: W2 = 0, b2 = const, W3 random: noise from layer-2 bias and layer-3 weights
torch.manual_seed(6)
a2 = learner.Actor().cuda()
with torch.no_grad():
    a2.l2.weight.zero_(); a2.l2.bias.uniform_(0.5, 1.5); a2.l3.weight.mul_(8); a2.l3.bias.zero_()
k2 = ActorKernel(a2, seed=4)
for sd in (0.05,):
    got = k2(x, noise_sd=sd)
    want = a2.forward_param_noise(x, sd, generator=torch.Generator(device="cuda").manual_seed(9))
    print(f"T2 W2=0 sd={sd}: kernel std {got.std(0).tolist()} torch std {want.std(0).tolist()}")
# T3: W1 = 0, b1 const
torch.manual_seed(7)
a3 = learner.Actor().cuda()
with torch.no_grad():
    a3.l1.weight.zero_(); a3.l1.bias.uniform_(0.5, 1.5); a3.l2.weight.mul_(4); a3.l3.weight.mul_(4)
k3 = ActorKernel(a3, seed=5)
got = k3(x, noise_sd=0.05)
want = a3.forward_param_noise(x, 0.05, generator=torch.Generator(device="cuda").manual_seed(9))
print(f"T3 W1=0 sd=0.05: kernel std {got.std(0).tolist()} torch std {want.std(0).tolist()}")

# learner loop sanity
L = learner.SkillshotLearner(n_envs=65536, seed=0, tick_limit=2000, replay_capacity=1 << 18)
obs = L.prepare_states()
print("obs finite", bool(torch.isfinite(obs).all()), "obs range", obs.min().item(), obs.max().item())
for t in range(60):
    act = L.model_act(obs)
    if t == 0:
        print("act finite", bool(torch.isfinite(act).all()), "abs mean", act.abs().mean().item(), "max", act.abs().max().item())
    out = L.do_actions(act)
    obs = out["obs_reset"]
g = L.game_environment
print("rot finite", bool(torch.isfinite(g.rot).all()), "counters", g.counters(), "live frac",
      g.game_live.float().mean().item(), "qvalid frac", g.projectile_valid.float().mean().item())
