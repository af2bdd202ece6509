"""The headline's own path at the headline's size:
bench.timed_ticks — the graph-replayed fused step over 65,536 games, seed 0,
random policy from the HBM action ring, random restarts — run for 2,100
timed ticks (plus its warm-up and capture launches, 2,600+ in all), so that
episodes cross the 2,000-tick limit and k_step's n >= 32,768 restart branch
(the early Philox draw, sk_engine.hip `kEarlyDrawMinEnvs`) runs.  The exact
launch sequence it executed (its trace) is replayed on libskillshot's CPU
backend (device = -1, csrc/sk_host.cpp, glibc trig) from the same start:
final state bit-exact, step counter and episode counters equal.  The
counters cover only the launches after the stream-ordered clear, so the
driver's `episodes` record is checked too (its race is the r02 finding)."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench_mod():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sys.path.insert(0, ROOT)
    import bench
    return bench


def _replay_on_cpu(ssa, start, acts, trace, n, tick_limit, seed):
    c = ssa.VecSkillshotGame(n, device="cpu", seed=seed, tick_limit=tick_limit)
    c.load_state_dict(start)
    ticks = 0
    for ev in trace:
        if ev[0] == "clear":
            c.clear_counters()
            continue
        s0, m = (0, ev[1]) if ev[0] == "run" else (ev[1], ev[2])
        c.step_multi(acts, n_ticks=m, slab0=s0)  # the launches for slabs s0 .. s0 + m - 1 (mod ring)
        ticks += m
    return c, ticks


@pytest.mark.parametrize("kind", ["k_step_graph", "multi"])
def test_bench_headline_path_equals_cpu_backend(bench_mod, kind):
    import skillshot_learning_amd as ssa
    dev = torch.device("cuda", 0)
    n, seed, limit, K, W, ring = 65536, 0, 2000, 2100, 5, 400
    trace = []
    if kind == "multi":
        el, ev, env = bench_mod.timed_multi(dev, n, seed, 0, limit, K, W, ring, 1, trace=trace)
    else:
        el, ev, env = bench_mod.timed_ticks(dev, n, seed, 0, limit, K, W, ring, 400, 1, trace=trace)
    torch.cuda.synchronize()
    got = env.state_dict()
    counters = env.counters()
    acts = env.bench_actions.cpu()
    # the start the bench stepped from: the same reset on a fresh engine
    start_env = ssa.VecSkillshotGame(n, device="cpu", seed=seed, tick_limit=limit)
    start_env.reset(random_positions=True)
    start = start_env.state_dict()
    # the action ring was generated after that reset, before any step
    c, ticks = _replay_on_cpu(ssa, start, acts, trace, n, limit, seed)
    assert ticks >= 2600 if kind == "k_step_graph" else ticks >= 2100
    want = c.state_dict()
    assert got.pop("step_counter") == want.pop("step_counter")
    for k in want:
        assert np.array_equal(np.asarray(got[k]), np.asarray(want[k])), k
    assert counters == c.counters()
    # episodes ended inside the counted launches only, and many crossed the limit
    assert counters["dones"] > n // 4 and counters["hits_p1"] + counters["hits_p2"] < counters["dones"]
    env.close()
