"""The in-launch exchange floor of a resident models_fit step (VERDICT r04
item 6; tools/seam_bench.hip): P workgroups on one XCD (S = 8) or spread
(S = 1) run R rounds of a critic step's three exchanges with nothing else,
for the two layer-2 partitions (rows: which 7 = all-gather + all-reduce +
reduce-scatter of 16 x 256; columns: which 56 = reduce-scatter of 16 x 128
partials + all-reduce + all-gather of 16 x 128; each alone beside); prints
one JSON line per configuration: us per round (HIP events over one launch of
R rounds) and the workgroups' XCC ids.

    python tools/seam_bench.py [--ps 4,8,16] [--rounds 2000]"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "ab_run", "libseam.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-fPIC", "-shared", "-std=c++17",
                    "-o", SO, os.path.join(ROOT, "tools", "seam_bench.hip")], check=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--ps", default="4,8,16")
    p.add_argument("--strides", default="8,1")
    p.add_argument("--rounds", type=int, default=2000)
    p.add_argument("--which", default="56,8,16,32,7")
    p.add_argument("--plain", default="0", help="0,1: also plain exchange stores (column partition, S = 8 only)")
    p.add_argument("--build", action="store_true")
    a = p.parse_args()
    if a.build:
        build()
        return
    L = ctypes.CDLL(SO)
    L.seam_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    xbuf = torch.zeros(2 * (16 * (512 + 16 + 4096) + 16 * 16 * 256 + 16 * 16 + 16 * 256), dtype=torch.int64,
                       device=dev)
    tmo = torch.zeros(1, dtype=torch.int32, device=dev)
    xcc = torch.zeros(64, dtype=torch.int32, device=dev)
    sink = torch.zeros(1, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev)
    epoch = [0]

    def run(P, S, R, which, plain):
        rc = L.seam_launch(xbuf.data_ptr(), tmo.data_ptr(), xcc.data_ptr(), sink.data_ptr(), P, S, R, epoch[0],
                           which, plain, ctypes.c_void_p(st.cuda_stream))
        assert rc == 0, rc
        epoch[0] += 3 * R + 3

    for P in [int(x) for x in a.ps.split(",")]:
        for S in [int(x) for x in a.strides.split(",")]:
            for which, plain in [(int(x), int(q)) for x in a.which.split(",") for q in a.plain.split(",")]:
                if plain and (S != 8 or which < 8):
                    continue
                run(P, S, 10, which, plain)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                run(P, S, a.rounds, which, plain)
                e1.record(st)
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.rounds
                names = {7: "rows A+Q+D", 1: "rows A", 2: "rows Q", 4: "rows D", 56: "cols R+Q2+G", 8: "cols R",
                         16: "cols Q2", 32: "cols G"}
                print(json.dumps(dict(P=P, S=S, which=names.get(which, which), stores="plain" if plain else "sc1",
                                      us_per_round=round(us, 3), timeout=int(tmo.item()),
                                      xcc=sorted(set(xcc[:P].tolist())))), flush=True)
                if int(tmo.item()):
                    sys.exit(3)


if __name__ == "__main__":
    main()
