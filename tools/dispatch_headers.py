"""Which AQL fence scopes does the HIP runtime put on k_step dispatches?

Run with AMD_LOG_LEVEL=4 (set by the caller): the runtime logs every packet
header ("Dispatch Header = 0x.. (type=2, barrier=b, acquire=a, release=r)"),
scope 0 none / 1 agent / 2 system.  Eager launches, then one replay of a
captured graph of 8 launches; the caller greps the log.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from skillshot_learning_amd import VecSkillshotGame  # noqa: E402

n = 65536
g = VecSkillshotGame(n, device="cuda:0", seed=0, random_positions=True)
st = torch.cuda.Stream()
with torch.cuda.stream(st):
    acts = g.gen_random_actions(8)
    done = torch.empty(n, dtype=torch.uint8, device="cuda:0")
st.synchronize()
sp = ctypes.c_void_p(st.cuda_stream)


def launch(t):
    g.step_raw(ctypes.c_void_p(acts.data_ptr() + t * 16 * n), ctypes.c_void_p(done.data_ptr()), stream=sp)


print("=== EAGER", flush=True)
with torch.cuda.stream(st):
    for t in range(4):
        launch(t)
st.synchronize()
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr, stream=st):
    for t in range(8):
        launch(t)
st.synchronize()
print("=== GRAPH REPLAY", flush=True)
with torch.cuda.stream(st):
    gr.replay()
st.synchronize()
print("=== END", flush=True)
