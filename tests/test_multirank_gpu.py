"""The multi-rank learner tick on the GPU (BASELINE configs 4 and 5 in
miniature): two ranks share the one GPU of the test box over gloo, each
steps its own shard of games (global ids rank * N ..), and the captured
learner tick (SkillshotLearner.tick_graph, "segmented" capture: graph
segments with the gloo collectives issued between them) all-reduces the
gradients ("grad") or all-gathers the sampled rows first ("shared").  The
ranks must hold identical nets after every replay; their games differ."""
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


def _worker(rank, world, port, mode, precision, overlap, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from skillshot_learning_amd.learner import SkillshotLearner
        n = 512
        L = SkillshotLearner(n_envs=n, device="cuda", seed=31, env_offset=rank * n, exploration="param_noise",
                             gamma=0.9, tau=0.05, replay_capacity=1 << 14, multi_rank=mode, precision=precision)
        tg = L.tick_graph(batch=64, ticks_per_graph=2, warmup=2, overlap=overlap)
        assert tg.multi_rank_mode == f"{mode}/segmented"
        # the reference-order tick by default; opted in, fp32 runs the fused
        # overlapped tick on every rank
        assert tg.mode == ("fused" if precision == "fp32" and overlap == "auto" else "sequential")
        tg.run(4)
        torch.cuda.synchronize()
        flat = torch.cat([p.detach().reshape(-1) for m in (L.model_actor, L.model_critic, L.ddpg.target_actor,
                                                            L.ddpg.target_critic) for p in m.parameters()]).cpu()
        pos = L.game_environment.pos.cpu()
        q.put((rank, flat.numpy(), pos.numpy(), int(L.replay.total_t)))
    except Exception as e:  # surface the failure to the parent
        import traceback
        q.put((rank, None, traceback.format_exc(), 0))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,precision,overlap", [("grad", "fp32", "0"), ("grad", "fp32", "auto"),
                                                    ("shared", "bf16", "0"), ("shared", "fp32", "auto")])
def test_two_rank_tick_graph_gloo(mode, precision, overlap):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import multiprocessing as mp
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, precision, overlap, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, flat, pos, total = q.get(timeout=300)
        assert flat is not None, pos
        out[rank] = (flat, pos, total)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.isfinite(out[0][0]).all()
    assert np.array_equal(out[0][0], out[1][0])       # identical nets after all-reduced updates
    assert not np.array_equal(out[0][1], out[1][1])   # different games on the two shards
    assert out[0][2] == out[1][2] > 0                 # each rank's ring took 2N rows per tick
