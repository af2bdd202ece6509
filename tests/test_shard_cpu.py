"""The engine's multi-GPU split on CPU with world_size-2 gloo:
games shard by contiguous global-id ranges and every RNG draw is keyed by the
global id, so two ranks each stepping their half (the oracle standing in for
the kernel, which the GPU tests hold bit-equal to it) reproduce one rank
stepping all games: identical state, and the episode counters all-reduced
over gloo equal the single-rank counters."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N, TICKS, LIMIT = 512, 300, 120


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _roll(n, offset, ticks):
    from oracle import oracle
    s = oracle.OracleState(n, seed=11, env_offset=offset)
    s.reset(random_positions=True)
    for _ in range(ticks):
        s.step(s.gen_random_actions(1)[0], tick_limit=LIMIT, auto_reset=True, random_positions=True, want_obs=False)
    return s


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = N // world
        s = _roll(n, rank * n, TICKS)
        c = torch.tensor([int(x) for x in s.counters[:4]], dtype=torch.int64)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        q.put((rank, {k: v.copy() for k, v in s.arrays().items()}, c.numpy()))
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_equal_one_rank():
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, arrays, counters = q.get(timeout=120)
        res[rank] = (arrays, counters)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole = _roll(N, 0, TICKS)
    ref = whole.arrays()
    for k, v in ref.items():
        got = np.concatenate([res[0][0][k], res[1][0][k]])
        assert np.array_equal(got.view(np.uint8), v.view(np.uint8)), k
    assert np.array_equal(res[0][1], res[1][1])
    assert np.array_equal(res[0][1], np.array([int(x) for x in whole.counters[:4]]))
    assert res[0][1][0] > 0  # episodes did end (and reset) inside the run
