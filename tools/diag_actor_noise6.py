import sys, ctypes, torch
sys.path.insert(0, "/root/repo")
from skillshot_learning_amd import learner
from skillshot_learning_amd.actor_kernel import ActorKernel
n = 200000
x = torch.zeros(n, 12, device="cuda")
a = learner.Actor().cuda()
with torch.no_grad():
    for l in (a.l1, a.l2, a.l3):
        l.weight.zero_(); l.bias.zero_()
    a.l1.bias[1] = 1.0; a.l2.weight[6, 1] = 1.0; a.l3.weight[1, 6] = 0.25   # chain B
    a.l1.bias[0] = 1.0; a.l2.weight[0, 0] = 1.0; a.l3.weight[0, 0] = 0.25   # chain 0
k = ActorKernel(a, seed=1)
L = k.L
L.skdiag_actor_forward_dbg.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_float, ctypes.c_uint64,
                                       ctypes.c_uint64, ctypes.c_void_p]
sd = 0.1
out = torch.empty(n, 2, device="cuda"); dbg = torch.zeros(n, 770, device="cuda")
L.skdiag_actor_forward_dbg(ctypes.c_void_p(k.buf.data_ptr()), ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                           ctypes.c_void_p(dbg.data_ptr()), n, sd, 7, 1, None)
torch.cuda.synchronize()
yd = torch.atanh(out.double()) / 0.25
yp = torch.atanh(k(x, noise_sd=sd).double()) / 0.25
print("debug build out var", yd.var(0).tolist(), " product build out var", yp.var(0).tolist(), " expect 0.0303 both")
print("debug: var h1_1 %.4f h2_6 %.4f pre3_1/0.25 %.4f corr(h1_1,h2_6) %.3f" % (dbg[:,1].var().item(), dbg[:,256+6].var().item(),
      (dbg[:,385]/0.25).var().item(), torch.corrcoef(torch.stack([dbg[:,1], dbg[:,256+6]]))[0,1].item()))
