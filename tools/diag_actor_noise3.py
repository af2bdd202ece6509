import sys, torch, math
sys.path.insert(0, "/root/repo")
from skillshot_learning_amd import learner
from skillshot_learning_amd.actor_kernel import ActorKernel
n = 400000
x = torch.zeros(n, 12, device="cuda")
a = learner.Actor().cuda()
with torch.no_grad():
    a.l1.weight.zero_(); a.l1.bias.zero_(); a.l2.weight.zero_(); a.l2.bias.zero_(); a.l3.weight.zero_(); a.l3.bias.zero_()
    a.l1.bias[0] = 1.0; a.l2.weight[0, 0] = 1.0; a.l3.weight[0, 0] = 0.25      # chain: unit 0 -> unit 0 -> out 0
    a.l1.bias[77] = 1.0; a.l2.weight[5, 77] = 1.0; a.l3.weight[1, 5] = 0.25    # chain: unit 77 -> unit 5 -> out 1
k = ActorKernel(a, seed=1)
for sd in (0.1, 0.3):
    y = torch.atanh(k(x, noise_sd=sd).double()) / 0.25
    ev = (1 + sd * sd) ** 3 - 1
    print(f"chain sd={sd}: mean {y.mean(0).tolist()} var {y.var(0).tolist()} expected mean ~1 var {ev:.5f}")
    t = a.forward_param_noise(x, sd, generator=torch.Generator(device="cuda").manual_seed(3))
    yt = torch.atanh(t.double()) / 0.25
    print(f"   torch: mean {yt.mean(0).tolist()} var {yt.var(0).tolist()}")
# mean path of the NOISE kernel: sd tiny vs deterministic kernel
torch.manual_seed(5)
b = learner.Actor().cuda()
with torch.no_grad():
    for l in (b.l1, b.l2, b.l3):
        l.weight.mul_(4.0); l.bias.normal_(0, 0.1)
kb = ActorKernel(b, seed=2)
xr = torch.rand(8192, 12, device="cuda")
d0 = kb(xr)
d1 = kb(xr, noise_sd=1e-7)
print("noise-kernel mean path vs deterministic kernel: max abs diff", (d0 - d1).abs().max().item())
