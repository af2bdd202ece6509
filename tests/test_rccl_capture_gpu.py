"""RCCL inside a captured learner tick, on the one GPU a test box has
(VERDICT r02 item 6): a world-size-1 NCCL (= RCCL) process group with the
multi-rank update forced on (DDPG force_collectives: the gradient all-reduce
of every update and, for multi_rank="shared", the minibatch all-gather), the
tick captured "full" (the collectives inside the hipGraph, the mode configs
4 and 5 take on an 8-GPU node) and "segmented" (the capture cut at every
collective, which is issued eagerly between the graph segments).  After 4
replays (8 ticks) both equal each other and the plain 1-rank tick graph
(no collectives) bit for bit: nets, target nets, Adam moments, game state.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def nccl_group():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    yield dist.group.WORLD
    dist.destroy_process_group()


def _run(mode, multi_rank, force, precision, tick="0"):
    from skillshot_learning_amd.learner import SkillshotLearner
    # one tick form for every run: the sequential one, or (fp32) the fused
    # overlapped one, which several ranks run too
    os.environ["SK_TICK_OVERLAP"] = tick
    if mode:
        os.environ["SK_TICKGRAPH_MODE"] = mode
    else:
        os.environ.pop("SK_TICKGRAPH_MODE", None)
    L = SkillshotLearner(n_envs=2048, device="cuda", seed=13, exploration="param_noise", gamma=0.99, tau=0.005,
                         replay_capacity=1 << 16, precision=precision, multi_rank=multi_rank,
                         force_collectives=force)
    tg = L.tick_graph(batch=256, ticks_per_graph=2, warmup=2)
    assert tg.mode == ("fused" if tick == "fused" else "sequential")
    got_mode = tg.multi_rank_mode
    tg.run(4)
    torch.cuda.synchronize()
    out = {}
    for name, m in (("actor", L.model_actor), ("critic", L.model_critic), ("t_actor", L.ddpg.target_actor),
                    ("t_critic", L.ddpg.target_critic)):
        for k, v in m.state_dict().items():
            out[f"{name}.{k}"] = v.detach().clone()
    fu = L.ddpg._fused
    out["adam_actor_m"] = fu.sa.m.clone()
    out["adam_critic_v"] = fu.sc.v.clone()
    for k, v in L.game_environment.state_dict().items():
        out[f"env.{k}"] = torch.as_tensor(v).clone()
    del tg, L
    os.environ.pop("SK_TICKGRAPH_MODE", None)
    os.environ.pop("SK_TICK_OVERLAP", None)
    return got_mode, out


@pytest.mark.parametrize("multi_rank,precision,tick", [("grad", "fp32", "0"), ("grad", "bf16", "0"),
                                                       ("shared", "fp32", "0"), ("shared", "bf16", "0"),
                                                       ("grad", "fp32", "fused"), ("shared", "fp32", "fused")])
def test_full_capture_equals_segmented_and_plain(nccl_group, multi_rank, precision, tick):
    mode_f, full = _run("full", multi_rank, True, precision, tick)
    mode_s, seg = _run("segmented", multi_rank, True, precision, tick)
    mode_p, plain = _run(None, multi_rank, False, precision, tick)
    assert mode_f == f"{multi_rank}/full" and mode_s == f"{multi_rank}/segmented" and mode_p is None
    for k in full:
        assert torch.equal(full[k], seg[k]), f"full vs segmented: {k}"
        assert torch.equal(full[k], plain[k]), f"full vs plain: {k}"
