"""Per-launch device time of each piece of one learner update, graph-replayed
(the way TickGraph runs them): K identical launches of one piece captured in
a hipGraph, HIP events around the replay, microseconds per launch.  Pieces:
replay sample, critic grad (bootstrap target in launch), critic Adam, actor
grad, actor Adam, and the whole update.  One JSON line per (precision, batch).

    python tools/bench_update_parts.py [--batches 256,4096] [--k 20] [--slices -1,0,1]

--slices sets SK_SLICE32 per pass (fp32: -1 automatic, 0 one-launch
gradient kernels, 1 the sliced two-launch schedule at every batch)."""
import argparse
import copy
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from skillshot_learning_amd.learner import DDPG  # noqa: E402


def timed(fn, st, k, reps=5):
    with torch.cuda.stream(st):
        for _ in range(2):
            fn()
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        for _ in range(k):
            fn()
    st.synchronize()
    best = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(st):
            e0.record()
            g.replay()
            e1.record()
        st.synchronize()
        best.append(e0.elapsed_time(e1) * 1e3 / k)
    best.sort()
    return round(best[len(best) // 2], 2)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batches", default="256,4096")
    p.add_argument("--k", type=int, default=20)
    p.add_argument("--precisions", default="fp32,bf16")
    p.add_argument("--slices", default="-1")
    p.add_argument("--w1-ablation", action="store_true")
    a = p.parse_args()
    for prec, sl, B in [(p_, s_, int(b)) for p_ in a.precisions.split(",") for s_ in a.slices.split(",")
                        for b in a.batches.split(",")]:
        if True:
            os.environ["SK_SLICE32"] = sl
            d = DDPG("cuda", seed=0, gamma=0.99, tau=0.005, replay_capacity=1 << 16, fused_update=True,
                     precision=prec)
            g = torch.Generator(device="cuda").manual_seed(0)
            n = 1 << 16
            s = torch.rand(n, 12, device="cuda", generator=g)
            d.replay.add(s, torch.rand(n, 2, device="cuda", generator=g) * 2 - 1,
                         torch.randn(n, device="cuda", generator=g), s.flip(0),
                         (torch.rand(n, device="cuda", generator=g) < 0.05).float())
            fu = d._fused
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                bs, ba, br, bs2, bd = d.sample_local(B, device_sampling=True)
            st.synchronize()
            pc = fu._partial(B, fu.fc.numel())
            pa = fu._partial(B, fu.fa.numel())
            out = dict(precision=prec, batch=B, k=a.k, slice=int(sl), sliced=pc.scratch is not None)
            out["sample"] = timed(lambda: d.sample_local(B, device_sampling=True), st, a.k)
            out["critic_grad"] = timed(lambda: fu._critic_grad(bs, ba, None, bs2, br, bd, 0.99, 0, B, pc,
                                                                fu.sc.steps, None), st, a.k)
            out["critic_adam"] = timed(lambda: fu._adam(pc, fu.fc, fu.sc, fu.tc, stat=fu.stats[0:1], scale=1.0 / B,
                                                        out=fu.loss_hist[0, 0], counter=fu.calls,
                                                        packs=fu._packs(critic=True)), st, a.k)
            if a.w1_ablation and pc.scratch is not None:
                # timing ablation (wrong gradients): the critic's Adam launch
                # summing 1/8 of the W1 / b1 contribution rows
                pc8 = copy.copy(pc)
                pc8.w1_rows = max(1, pc.w1_rows // 8)
                out["critic_adam_w1_rows_div8"] = timed(
                    lambda: fu._adam(pc8, fu.fc, fu.sc, fu.tc, stat=fu.stats[0:1], scale=1.0 / B,
                                     out=fu.loss_hist[0, 0], counter=fu.calls, packs=fu._packs(critic=True)), st, a.k)
            out["actor_grad"] = timed(lambda: fu._actor_grad(bs, pa, fu.sa.steps, fu.stats[1:]), st, a.k)
            out["actor_adam"] = timed(lambda: fu._adam(pa, fu.fa, fu.sa, fu.ta, stat=fu.stats[1:], scale=-1.0,
                                                       out=fu.loss_hist[1, 0], packs=fu._packs(critic=False)),
                                      st, a.k)
            out["update"] = timed(lambda: d.replay_update(B, device_sampling=True), st, a.k)
            out["sum_of_pieces"] = round(sum(out[k] for k in ("sample", "critic_grad", "critic_adam", "actor_grad",
                                                                "actor_adam")), 2)
            print(json.dumps(out), flush=True)
            del d, fu
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
