import torch, json
torch.cuda.init()
res = {}
for mb in (405, 1024):
    n = mb * (1 << 20) // 4
    a = torch.empty(n, device="cuda"); b = torch.empty(n, device="cuda"); a.fill_(1.0)
    for _ in range(3): b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): b.copy_(a)
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    res[f"copy_{mb}MB"] = dict(us=us, tbs=2 * n * 4 / (us * 1e-6) / 1e12)
    e0.record()
    for _ in range(20): a.sum()
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    res[f"read_{mb}MB"] = dict(us=us, tbs=n * 4 / (us * 1e-6) / 1e12)
    e0.record()
    for _ in range(20): b.fill_(2.0)
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    res[f"write_{mb}MB"] = dict(us=us, tbs=n * 4 / (us * 1e-6) / 1e12)
print(json.dumps(res))
