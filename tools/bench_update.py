"""Device time of one learner update (critic step with in-launch bootstrap
target + actor step, Keras Adam, soft update) at both precisions, per batch
size: mean over --iters updates replayed from a captured hipGraph, HIP
events on the graph's stream.  One JSON line per (precision, batch)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from skillshot_learning_amd.learner import DDPG  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batches", default="256,4096")
    p.add_argument("--iters", type=int, default=200)
    a = p.parse_args()
    for prec in ("fp32", "bf16"):
        for B in [int(x) for x in a.batches.split(",")]:
            d = DDPG("cuda", seed=0, gamma=0.99, tau=0.005, replay_capacity=1 << 16, fused_update=True,
                     precision=prec)
            g = torch.Generator(device="cuda").manual_seed(0)
            s = torch.rand(1 << 16, 12, device="cuda", generator=g)
            d.replay.add(s, torch.rand(1 << 16, 2, device="cuda", generator=g) * 2 - 1,
                         torch.randn(1 << 16, device="cuda", generator=g), s.flip(0),
                         (torch.rand(1 << 16, device="cuda", generator=g) < 0.05).float())
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                for _ in range(3):
                    d.replay_update(B, device_sampling=True)
            st.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=st):
                for _ in range(10):
                    d.replay_update(B, device_sampling=True)
            st.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(st):
                gr.replay()
                e0.record()
                for _ in range(a.iters // 10):
                    gr.replay()
                e1.record()
            st.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / ((a.iters // 10) * 10)
            print(json.dumps(dict(precision=prec, batch=B, us_per_update=us,
                                  note="replay sample + critic step (bootstrap in launch) + Adam + actor step + Adam")),
                  flush=True)
            del gr, d
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
