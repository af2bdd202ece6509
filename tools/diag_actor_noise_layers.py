"""Per-layer moments of the noisy actor kernel (debug entry dumps every unit)
against the torch local-reparameterisation reference, in the setting of
tests/test_actor_gpu.py::test_param_noise_kernel_distribution."""
import ctypes
import sys

import torch

sys.path.insert(0, "/root/repo")
from skillshot_learning_amd import learner
from skillshot_learning_amd.actor_kernel import ActorKernel

torch.manual_seed(5)
a = learner.Actor().cuda()
with torch.no_grad():
    for l in (a.l1, a.l2, a.l3):
        l.weight.mul_(4.0)
        l.bias.normal_(0, 0.1)
n, sd = 200000, 0.5
x = torch.rand(1, 12, device="cuda").expand(n, 12).contiguous()
k = ActorKernel(a, seed=11)
L = k.L
L.skdiag_actor_forward_dbg.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_float, ctypes.c_uint64,
                                                                 ctypes.c_uint64, ctypes.c_void_p]
out = torch.empty(n, 2, device="cuda")
dbg = torch.zeros(n, 770, device="cuda")
L.skdiag_actor_forward_dbg(ctypes.c_void_p(k.buf.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                           ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(dbg.data_ptr()), n, sd, 7, 1, None)
torch.cuda.synchronize()

g = torch.Generator(device="cuda").manual_seed(2)
ref = []
h = x
for i, l in enumerate((a.l1, a.l2, a.l3)):
    m = torch.nn.functional.linear(h, l.weight, l.bias)
    v = torch.nn.functional.linear(h * h, l.weight * l.weight, l.bias * l.bias)
    y = m + sd * v.clamp_min(0).sqrt() * torch.randn(m.shape, device="cuda", generator=g)
    ref.append(y if i == 2 else torch.relu(y))
    h = ref[-1]
segs = [(0, 256), (256, 384), (384, 386)]
for i, (lo, hi) in enumerate(segs):
    kd, rd = dbg[:, lo:hi].double(), ref[i].double()
    km, rm, ks, rs = kd.mean(0), rd.mean(0), kd.std(0), rd.std(0)
    z = (km - rm).abs() / (rs / n ** 0.5 + 1e-12)
    ratio = ks / (rs + 1e-12)
    live = rs > 1e-6
    print(f"layer {i + 1}: units {hi - lo}  mean-diff z max {z[live].max():.1f} med {z[live].median():.2f}  "
          f"std ratio min {ratio[live].min():.3f} max {ratio[live].max():.3f} med {ratio[live].median():.4f}")
    worst = int(torch.argmax(torch.where(live, z, torch.zeros_like(z))))
    print(f"   worst unit {worst}: kernel mean {km[worst]:.4f} std {ks[worst]:.4f}  ref mean {rm[worst]:.4f} "
          f"std {rs[worst]:.4f}")
# layer-2 units recomputed from the kernel's own layer-1 dump (isolates layer 2)
h1 = dbg[:, :256]
m = torch.nn.functional.linear(h1, a.l2.weight, a.l2.bias)
v = torch.nn.functional.linear(h1 * h1, a.l2.weight ** 2, a.l2.bias ** 2)
y2 = torch.relu(m + sd * v.clamp_min(0).sqrt() * torch.randn(m.shape, device="cuda", generator=g)).double()
kd = dbg[:, 256:384].double()
z = (kd.mean(0) - y2.mean(0)).abs() / (y2.std(0) / n ** 0.5 + 1e-12)
ratio = kd.std(0) / (y2.std(0) + 1e-12)
live = y2.std(0) > 1e-6
print(f"layer 2 | kernel h1: mean-diff z max {z[live].max():.1f} med {z[live].median():.2f} "
      f"std ratio min {ratio[live].min():.3f} max {ratio[live].max():.3f}")
h2 = dbg[:, 256:384]
m = torch.nn.functional.linear(h2, a.l3.weight, a.l3.bias)
v = torch.nn.functional.linear(h2 * h2, a.l3.weight ** 2, a.l3.bias ** 2)
y3 = (m + sd * v.clamp_min(0).sqrt() * torch.randn(m.shape, device="cuda", generator=g)).double()
kd = dbg[:, 384:386].double()
print("layer 3 | kernel h2: kernel mean/std", kd.mean(0).tolist(), kd.std(0).tolist(), " ref", y3.mean(0).tolist(),
      y3.std(0).tolist())
# correlations between layer-1 units in the kernel (should be ~0 for distinct units)
c = torch.corrcoef(dbg[:20000, :256].T.double())
c = c[torch.isfinite(c)]
off = c[(c.abs() < 0.999)]
print(f"layer-1 |corr| between units: max {off.abs().max():.3f} mean {off.abs().mean():.4f}")

# ---- layer 2 internals: mean accumulator, variance accumulator, normals
bf = lambda t: t.to(torch.bfloat16).float()
h1b = bf(dbg[:4096, :256])
acc_ref = h1b @ bf(a.l2.weight).t()
var_ref = bf(h1b * h1b) @ bf(a.l2.weight ** 2).t()
acc_k, var_k, z_k = dbg[:4096, 386:514], dbg[:4096, 514:642], dbg[:, 642:770].double()
print(f"layer-2 acc: max |diff| {(acc_k - acc_ref).abs().max():.3e} (scale {acc_ref.abs().max():.2f})")
rel = (var_k - var_ref).abs() / var_ref.abs().clamp_min(1e-6)
print(f"layer-2 var: median rel diff {rel.median():.3e} max {rel.max():.3e}; kernel/ref mean ratio "
      f"{(var_k.mean(0) / var_ref.mean(0).clamp_min(1e-9)).median():.4f}")
zm, zv = z_k.mean(0), z_k.var(0)
print(f"layer-2 z: per-unit mean |max| {zm.abs().max():.4f}  var min {zv.min():.4f} max {zv.max():.4f} "
      f"mean {zv.mean():.4f}")
cz = torch.corrcoef(z_k[:20000].T)
offd = cz[~torch.eye(128, dtype=torch.bool, device=cz.device)]
print(f"layer-2 z corr between units: max |c| {offd.abs().max():.4f}")
hist = torch.histc(z_k[:, 0].float(), bins=12, min=-3, max=3)
print("z[:,0] histogram (-3..3, 12 bins):", [int(v) for v in hist.tolist()])

import os
os.makedirs("gpurun_out", exist_ok=True)
torch.save(dict(dbg=dbg[:4096].cpu(), x=x[:1].cpu(), sd=sd,
                w={k: v.detach().cpu() for k, v in a.state_dict().items()}), "gpurun_out/diag7_dump.pt")
