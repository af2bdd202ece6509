"""Device time of the actor forward kernels (fp32 sk_actor_forward_f32, bf16
sk_actor_forward_advance) with and without parameter noise, per row count
(rows = 2 x games: both players), HIP events around one replay of a hipGraph
of --iters launches (no host launch time).  --fwd16 sets SK_FWD16 per pass
(fp32: -1 automatic, 0 the 32-row kernel, 1 the 16-row kernel)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from skillshot_learning_amd.actor_kernel import ActorKernel, ActorKernel32  # noqa: E402
from skillshot_learning_amd.learner import Actor  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", default="8192,131072")
    p.add_argument("--iters", type=int, default=50)
    p.add_argument("--fwd16", default="-1")
    p.add_argument("--precisions", default="fp32,bf16")
    a = p.parse_args()
    torch.manual_seed(0)
    actor = Actor().cuda()
    kernels = {"fp32": ActorKernel32(actor, seed=1), "bf16": ActorKernel(actor, seed=1)}
    st = torch.cuda.Stream()
    for f16 in a.fwd16.split(","):
        os.environ["SK_FWD16"] = f16
        for rows in [int(r) for r in a.rows.split(",")]:
            x = torch.rand(rows, 12, device="cuda")
            out = torch.empty(rows, 2, device="cuda")
            for prec in a.precisions.split(","):
                k = kernels[prec]
                for sd, asd in ((0.0, 0.0), (0.5, 0.0), (0.0, 0.15)):
                    st.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(st):
                        for _ in range(3):
                            k(x, noise_sd=sd, out=out, action_sd=asd)
                    st.synchronize()
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=st):
                        for _ in range(a.iters):
                            k(x, noise_sd=sd, out=out, action_sd=asd)
                    ts = []
                    for _ in range(3):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        with torch.cuda.stream(st):
                            e0.record()
                            g.replay()
                            e1.record()
                        st.synchronize()
                        ts.append(e0.elapsed_time(e1) * 1e3 / a.iters)
                    us = sorted(ts)[1]
                    flop = 72192 * rows * (2 if sd else 1)  # 2 x MACs of 12x256 + 256x128 + 128x2; noise doubles
                    print(json.dumps(dict(precision=prec, fwd16=int(f16), rows=rows, param_noise=sd, action_noise=asd,
                                          us=round(us, 2), tflops=round(flop / (us * 1e-6) / 1e12, 1))), flush=True)


if __name__ == "__main__":
    main()
