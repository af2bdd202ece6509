"""BASELINE configs 4 and 5 at their per-rank workloads on the GPU (VERDICT
r04 item 1, r05 item 4): two ranks share the one GPU of the test box over
gloo, each rank a fresh process holding its config's share of games.

  config 4: 32,768 games over 8 GPUs = 4,096 per rank, multi_rank="grad"
            (each rank samples its own ring, gradient all-reduce), action
            noise, batch 256, fp32;
  config 5: 65,536 games over 8 GPUs = 8,192 per rank, multi_rank="shared"
            (the ranks' samples all-gathered, rank r steps rows r::world),
            parameter noise, batch 256, fp32.

Each rank runs the captured learner tick (reference order, "segmented"
capture: graph segments with the gloo collectives issued between them; one
tick per graph, so the odd-count phase graphs run too) for 20 ticks,
recording each tick's actions, then ONE update through the replay rule's own
sampled path (DDPG.update_sampled: grad draws from this rank's ring inside
the critic launch; shared draws, all-gathers and steps rows r::world), and
returns the rows it drew.  Asserted:
  * the ranks' nets (online and target) are identical after the replays and
    after the update; their games differ;
  * each rank's shard after the 20 ticks equals a one-rank VecSkillshotGame
    over the same global env ids (CPU backend, the same start state and the
    recorded actions), bit for bit: the shards need no exchange;
  * the sharded update equals the ONE-rank fused update on exactly the rows
    the ranks drew, concatenated in the order the ranks numbered them, from
    the same starting state (nets, target nets, Adam moments and steps,
    Dropout call number) within 1e-5 — the GPU analogue of
    tests/test_learner_keras_cpu.py::test_two_ranks_equal_one_rank_on_concatenated_batch;
  * the same update against the fp64 Keras restatement (oracle/keras_ref.py)
    on those rows within 1e-5 (parity unpinned against Keras itself:
    TensorFlow is absent).
Reference: SkillshotLearner.py:419-443 (the update), SkillshotGame.py:58-94
(games are independent, so the shards need no exchange)."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

PARAM_ABS = 1e-5  # parameters after one Adam step (1 % of an lr-sized step)
CFGS = {"config4": (4096, "grad", "action_noise"), "config5": (8192, "shared", "param_noise")}
BATCH = 256
NETS = ("fa", "fc", "ta", "tc")
TICKS = 20


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _state(d):
    fu = d._fused
    t = dict(fa=fu.fa, fc=fu.fc, ta=fu.ta, tc=fu.tc, am=fu.sa.m, av=fu.sa.v, ast=fu.sa.steps, cm=fu.sc.m,
             cv=fu.sc.v, cst=fu.sc.steps, calls=d.drop_calls)
    return {k: v.detach().cpu().numpy().copy() for k, v in t.items()}


def _worker(rank, world, port, cfg, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from skillshot_learning_amd.learner import SkillshotLearner
        n, mode, expl = CFGS[cfg]
        L = SkillshotLearner(n_envs=n, device="cuda", seed=41, env_offset=rank * n, exploration=expl, gamma=0.9,
                             tau=0.05, replay_capacity=1 << 20, multi_rank=mode, precision="fp32")
        assert L.ddpg._fused is not None and L.ddpg._fused.f32
        tg = L.tick_graph(batch=BATCH, ticks_per_graph=1, warmup=2)
        assert tg.multi_rank_mode == f"{mode}/segmented" and tg.mode == "sequential"
        g = L.game_environment
        torch.cuda.synchronize()
        st0 = g.state_dict()
        acts = []
        for _ in range(TICKS):
            tg.run(1)
            acts.append(tg.act.detach().cpu().numpy().copy())
        torch.cuda.synchronize()
        st1 = g.state_dict()
        d = L.ddpg
        before = _state(d)
        d.update_sampled(BATCH)  # the replay rule's own draw (grad: own ring in-launch; shared: drawn + gathered)
        torch.cuda.synchronize()
        # numpy, not tensors: a CPU tensor crosses the queue as a shared-memory fd
        # that dies with this process, which may exit before the parent reads it
        rows = [t.detach().cpu().numpy().copy() for t in L.replay._batch_bufs(BATCH)]
        after = _state(d)
        q.put((rank, before, after, int(L.replay.total_t), rows, st0, st1, acts, g.tick_limit))
    except Exception:  # surface the failure to the parent
        import traceback
        q.put((rank, None, traceback.format_exc(), 0, None, None, None, None, 0))
        raise
    finally:
        dist.destroy_process_group()


def _shard_replay(rank, n, st0, acts, tick_limit):
    """the shard's games on their own: a one-rank VecSkillshotGame over global
    env ids rank*n .. rank*n + n - 1 (CPU backend), from the shard's start
    state, stepped with the recorded actions (auto-reset, random starts)"""
    from skillshot_learning_amd.vec_env import VecSkillshotGame
    env = VecSkillshotGame(n, device="cpu", seed=41, env_offset=rank * n, tick_limit=tick_limit,
                           random_positions=True)
    env.load_state_dict(st0)
    for a in acts:
        env.step(torch.from_numpy(a), obs=False, auto_reset=True)
    out = env.state_dict()
    env.close()
    return out


def _one_rank_update(state, rows):
    """the fused fp32 update of ONE rank from `state` on the concatenated rows"""
    from skillshot_learning_amd.learner import DDPG
    d = DDPG("cuda", seed=41, gamma=0.9, tau=0.05, fused_update=True, precision="fp32")
    fu = d._fused
    with torch.no_grad():
        for k, t in dict(fa=fu.fa, fc=fu.fc, ta=fu.ta, tc=fu.tc, am=fu.sa.m, av=fu.sa.v, ast=fu.sa.steps,
                         cm=fu.sc.m, cv=fu.sc.v, cst=fu.sc.steps, calls=d.drop_calls).items():
            t.copy_(torch.from_numpy(state[k]))
    fu.pack()
    d.update_batch(*rows)
    torch.cuda.synchronize()
    return d, _state(d)


def _keras_update(d0, state, rows):
    """the same update restated in fp64 (oracle/keras_ref.py): bootstrap
    target from the target nets, critic step, actor step on the stepped
    critic, Keras Adam from the loaded moments, soft update"""
    from oracle import keras_ref as kr
    from skillshot_learning_amd import rng

    def unflat(flat, module):
        out, off = {}, 0
        for name, p in module.named_parameters():
            out[name] = flat[off:off + p.numel()].astype(np.float64).reshape(tuple(p.shape))
            off += p.numel()
        return out

    def adam(P, module, m, v, steps):  # Keras Adam resumed from the loaded moments and step count
        o = kr.Adam(P)
        o.m, o.v = unflat(m, module), unflat(v, module)
        assert len(set(steps.tolist())) == 1
        o.t = int(steps[0])
        return o

    A, C = unflat(state["fa"], d0.model_actor), unflat(state["fc"], d0.model_critic)
    TA, TC = unflat(state["ta"], d0.model_actor), unflat(state["tc"], d0.model_critic)
    oa = adam(A, d0.model_actor, state["am"], state["av"], state["ast"])
    oc = adam(C, d0.model_critic, state["cm"], state["cv"], state["cst"])
    s, a, r, s2, dn = [t.double().cpu().numpy() for t in rows]
    B = s.shape[0]
    keep = rng.dropout_keep(d0.drop_seed, int(state["calls"][0]), 0, B).double().numpy()
    y = kr.target_y(TA, TC, s2, r, dn, 0.9)
    gc, _ = kr.critic_grads(C, s, a, y, keep)
    C = oc.step(C, gc)
    ga, _ = kr.actor_grads(A, C, s)
    A = oa.step(A, ga)
    TA, TC = kr.soft_update(TA, A, 0.05), kr.soft_update(TC, C, 0.05)

    def flat(P, module):
        return np.concatenate([P[name].reshape(-1) for name, _ in module.named_parameters()])
    return dict(fa=flat(A, d0.model_actor), fc=flat(C, d0.model_critic), ta=flat(TA, d0.model_actor),
                tc=flat(TC, d0.model_critic))


@pytest.mark.parametrize("cfg", list(CFGS))
def test_config_per_rank_workload_two_ranks(cfg):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import multiprocessing as mp
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, before, after, total, rows, st0, st1, acts, lim = q.get(timeout=600)
            assert before is not None, after
            out[rank] = (before, after, total, rows, st0, st1, acts, lim)
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
    finally:  # never leave a rank behind (the interpreter would wait for it at exit)
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=30)
    b0, a0, t0 = out[0][:3]
    b1, a1, t1 = out[1][:3]
    n, mode, _ = CFGS[cfg]
    # identical nets (and Adam state) on both ranks after the replays and after the update
    for k in b0:
        assert np.array_equal(b0[k], b1[k]), ("before", k)
        assert np.array_equal(a0[k], a1[k]), ("after", k)
    assert np.isfinite(a0["fa"]).all() and np.isfinite(a0["fc"]).all()
    assert t0 == t1 > 0
    assert not np.array_equal(out[0][5]["pos"], out[1][5]["pos"])  # different games on the two shards
    assert int(a0["calls"][0]) == int(b0["calls"][0]) + 1  # one critic step's Dropout call
    # each shard equals its games run alone over the same global env ids
    for r in range(world):
        _, _, _, _, st0, st1, acts, lim = out[r]
        assert st1["pos"].shape[0] == n and len(acts) == TICKS
        want = _shard_replay(r, n, st0, acts, lim)
        for k in want:
            assert np.array_equal(np.asarray(want[k]), np.asarray(st1[k])), (cfg, r, k)
    # the one-rank update on exactly the rows the ranks drew (rank order)
    full = [torch.cat([torch.from_numpy(out[r][3][j]) for r in range(world)]).to("cuda") for j in range(5)]
    if mode == "shared":  # rank r stepped rows r::world of the gathered batch
        full = [torch.cat([t[r::world] for r in range(world)]) for t in full]
    d1, want = _one_rank_update(b0, full)
    for k in NETS:
        err = np.abs(a0[k] - want[k]).max()
        assert err <= PARAM_ABS, (cfg, k, err)
        assert not np.array_equal(a0[k], b0[k]), (cfg, k)  # the update moved every net
    # and against the fp64 Keras restatement on those rows
    ref = _keras_update(d1, b0, full)
    for k in NETS:
        err = np.abs(a0[k] - ref[k]).max()
        assert err <= PARAM_ABS, (cfg, "keras", k, err)
