import sys, ctypes, torch
sys.path.insert(0, "/root/repo")
from skillshot_learning_amd import learner
from skillshot_learning_amd.actor_kernel import ActorKernel
n = 100000
x = torch.zeros(n, 12, device="cuda")
a = learner.Actor().cuda()
with torch.no_grad():
    for l in (a.l1, a.l2, a.l3):
        l.weight.zero_(); l.bias.zero_()
    a.l1.bias.fill_(1.0)                       # every layer-1 unit = relu(1 + sd*xi): var sd^2
    a.l2.weight[torch.arange(128), torch.arange(128)] = 1.0   # layer-2 unit j = relu(h1_j (1 + sd*xi))
k = ActorKernel(a, seed=1)
L = k.L
L.skdiag_actor_forward_dbg.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_float, ctypes.c_uint64,
                                       ctypes.c_uint64, ctypes.c_void_p]
out = torch.empty(n, 2, device="cuda")
dbg = torch.zeros(n, 386, device="cuda")
sd = 0.1
rc = L.skdiag_actor_forward_dbg(ctypes.c_void_p(k.buf.data_ptr()), ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                ctypes.c_void_p(dbg.data_ptr()), n, sd, 7, 1, None)
torch.cuda.synchronize()
v1 = dbg[:, :256].var(0)
v2 = dbg[:, 256:384].var(0)
print("L1 unit var (expect 0.01): min %.4f max %.4f" % (v1.min().item(), v1.max().item()))
bad1 = (v1 < 0.008).nonzero().flatten().tolist()
print("L1 bad units:", bad1[:40], len(bad1))
print("L2 unit var (expect (1.01)^2-1=0.0201): min %.4f max %.4f" % (v2.min().item(), v2.max().item()))
bad2 = ((v2 < 0.017) | (v2 > 0.024)).nonzero().flatten().tolist()
print("L2 bad units:", bad2[:40], len(bad2))
c = torch.corrcoef(torch.stack([dbg[:, 1], dbg[:, 256 + 1], dbg[:, 6], dbg[:, 256 + 6], dbg[:, 0], dbg[:, 256]]))
print("corr (h1_1, h2_1, h1_6, h2_6, h1_0, h2_0):\n", c)
