"""Two RCCL ranks on two GPUs: the multi-rank learner
tick captured "full" (the gradient all-reduce / shared-replay all-gather
inside the hipGraph), for multi_rank "grad" (config 4) and "shared"
(config 5), in the reference-order tick and the opt-in fused overlapped one.
Both ranks must hold identical nets after every update, different games on
their shards, and equal ring counts; and the full capture must equal the
segmented one (collectives issued between graph segments) bit for bit.
Skipped unless the box has at least two GPUs (the driver's 8-GPU node runs
it; a one-GPU box skips it)."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, mode, precision, overlap, capture, q):
    import datetime

    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["SK_TICKGRAPH_MODE"] = capture
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank),
                            timeout=datetime.timedelta(seconds=120))
    try:
        from skillshot_learning_amd.learner import SkillshotLearner
        n = 2048
        L = SkillshotLearner(n_envs=n, device=f"cuda:{rank}", seed=41, env_offset=rank * n,
                             exploration="param_noise" if mode == "shared" else "action_noise", gamma=0.99,
                             tau=0.005, replay_capacity=1 << 16, multi_rank=mode, precision=precision)
        tg = L.tick_graph(batch=256, ticks_per_graph=2, warmup=2, overlap=overlap)
        assert tg.multi_rank_mode == f"{mode}/{capture}"
        tg.run(4)
        torch.cuda.synchronize()
        flat = torch.cat([p.detach().reshape(-1) for m in (L.model_actor, L.model_critic, L.ddpg.target_actor,
                                                            L.ddpg.target_critic) for p in m.parameters()]).cpu()
        q.put((rank, flat.numpy(), L.game_environment.pos.cpu().numpy(), int(L.replay.total_t), tg.mode))
    except Exception:  # surface the failure to the parent
        import traceback
        q.put((rank, None, traceback.format_exc(), 0, None))
        raise
    finally:
        dist.destroy_process_group()


def _run(mode, precision, overlap, capture):
    import multiprocessing as mp
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, precision, overlap, capture, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, flat, pos, total, tmode = q.get(timeout=240)
            assert flat is not None, pos
            out[rank] = (flat, pos, total, tmode)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return out


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2, reason="needs two GPUs")
@pytest.mark.parametrize("mode,precision,overlap", [("grad", "fp32", "0"), ("grad", "fp32", "auto"),
                                                    ("shared", "fp32", "0"), ("shared", "fp32", "auto"),
                                                    ("shared", "bf16", "0")])
def test_two_rccl_ranks_full_capture(mode, precision, overlap):
    full = _run(mode, precision, overlap, "full")
    assert np.isfinite(full[0][0]).all()
    assert np.array_equal(full[0][0], full[1][0])        # identical nets after all-reduced updates
    assert not np.array_equal(full[0][1], full[1][1])    # different games on the two shards
    assert full[0][2] == full[1][2] > 0
    assert full[0][3] == ("fused" if precision == "fp32" and overlap == "auto" else "sequential")
    seg = _run(mode, precision, overlap, "segmented")
    for r in (0, 1):
        assert np.array_equal(full[r][0], seg[r][0])     # RCCL in the graph == RCCL between segments
        assert np.array_equal(full[r][1], seg[r][1])
