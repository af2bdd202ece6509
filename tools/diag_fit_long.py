"""Resident critic pass vs the three-launch chain over long passes (ADVICE
r05): is the parting of the two fp32 trajectories chaotic (relu flips
amplifying two summation orders) or a bias of the resident kernel's
arithmetic (its v_rcp_f32(v_sqrt_f32(v) + eps) Adam, its tanh)?

For each pass length n, from the same start and rows, max |parameter
difference| of:
  err_per{4096,2048,512}  the resident pass (cut into launches of that many
                          steps) against the chain (launch cuts change
                          nothing: the same bits);
  resident_vs_fp64,       each fp32 path against the fp64 Keras restatement
  chain_vs_fp64           (oracle/keras_ref.py, the same Dropout keys);
  chain_vs_chain_ulp      the chain against itself started with ONE
                          parameter moved by one ulp: the spread any fp32
                          implementation's rounding produces.
If resident_vs_fp64 ~ chain_vs_fp64 and err ~ chain_vs_chain_ulp, the two
paths are equally valid trajectories of a chaotic map.

    python tools/diag_fit_long.py [--ns 256,1024,2040,2600]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="256,1024,2040,2600")
    args = ap.parse_args()
    from oracle import keras_ref as kr
    from skillshot_learning_amd import learner, rng
    dev = torch.device("cuda", 0)

    def rows(n, seed):
        g = torch.Generator(device=dev).manual_seed(seed)
        s = torch.rand(16 * n, 12, device=dev, generator=g) * torch.tensor(
            [1, 1, 1, 1, 9.8, 1, 1, 1, 1, 9.8, 1, 1.0], device=dev)
        return s, torch.rand(16 * n, 2, device=dev, generator=g) * 2 - 1, torch.randn(16 * n, device=dev,
                                                                                       generator=g) * 0.5

    def chain(n, s, a, y, ulp=False):
        d = learner.DDPG("cuda", seed=6, fused_update=True, precision="fp32")
        if ulp:  # one parameter one ulp up (the first W2 entry)
            with torch.no_grad():
                f = d._fused.fc
                i = 256 * 12 + 256
                f[i] = torch.nextafter(f[i], torch.tensor(float("inf"), device=f.device))
        for k in range(n):
            d.critic_step(s[16 * k:16 * k + 16], a[16 * k:16 * k + 16], y[16 * k:16 * k + 16])
        torch.cuda.synchronize()
        return d

    for n in [int(x) for x in args.ns.split(",")]:
        s, a, y = rows(n, 13)
        out = dict(n=n)
        ref = chain(n, s, a, y)
        ref_fc = ref._fused.fc.double().cpu().numpy()
        for per in (4096, 2048, 512):
            d = learner.DDPG("cuda", seed=6, fused_update=True, precision="fp32")
            d._fused.FIT_STEPS_PER_LAUNCH = per
            d._fused.fit_critic(s, a, y)
            d._fused.fit_check()
            torch.cuda.synchronize()
            out[f"err_per{per}"] = (d._fused.fc - ref._fused.fc).abs().max().item()
            out[f"steps_eq_per{per}"] = bool(torch.equal(d._fused.sc.steps, ref._fused.sc.steps))
            if per == 4096:
                res_fc = d._fused.fc.double().cpu().numpy()
        pert = chain(n, s, a, y, ulp=True)
        out["chain_vs_chain_ulp"] = float(np.abs(pert._fused.fc.double().cpu().numpy() - ref_fc).max())
        # the fp64 restatement from the same start, step by step
        d0 = learner.DDPG("cuda", seed=6, fused_update=True, precision="fp32")
        C = kr.from_module(d0.model_critic)
        call0 = int(d0.drop_calls)
        oc = kr.Adam(C)
        sn, an, yn = [t.double().cpu().numpy() for t in (s, a, y)]
        for k in range(n):
            sl = slice(16 * k, 16 * k + 16)
            keep = rng.dropout_keep(d0.drop_seed, call0 + k, 0, 16).double().numpy()
            gc, _ = kr.critic_grads(C, sn[sl], an[sl], yn[sl], keep)
            C = oc.step(C, gc)
        f64 = np.concatenate([C[name].reshape(-1) for name, _ in d0.model_critic.named_parameters()])
        out["resident_vs_fp64"] = float(np.abs(res_fc - f64).max())
        out["chain_vs_fp64"] = float(np.abs(ref_fc - f64).max())
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
