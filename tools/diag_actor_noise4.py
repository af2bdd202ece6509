import sys, torch
sys.path.insert(0, "/root/repo")
from skillshot_learning_amd import learner
from skillshot_learning_amd.actor_kernel import ActorKernel
n = 400000
x = torch.zeros(n, 12, device="cuda")
a = learner.Actor().cuda()
with torch.no_grad():
    for l in (a.l1, a.l2, a.l3):
        l.weight.zero_(); l.bias.zero_()
    a.l1.bias[4] = 1.0; a.l2.weight[0, 4] = 1.0; a.l3.weight[0, 0] = 0.25   # A: L1 h=1 -> L2 h=0
    a.l1.bias[1] = 1.0; a.l2.weight[6, 1] = 1.0; a.l3.weight[1, 6] = 0.25   # B: L1 h=0 -> L2 h=1
k = ActorKernel(a, seed=1)
sd = 0.1
y = torch.atanh(k(x, noise_sd=sd).double()) / 0.25
print("A (L1 h=1, L2 h=0) var", y.var(0)[0].item(), " B (L1 h=0, L2 h=1) var", y.var(0)[1].item(),
      " all-three 0.0303, two 0.0201, one 0.0100")
