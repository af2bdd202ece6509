"""BASELINE config 3 on the GPU: 4,096 games + DDPG (actor with action noise,
fused env step with obs/reward/auto-reset, 1 M-row replay ring in HBM,
minibatch 256, one critic + actor update per tick), replayed as captured
learner ticks (SkillshotLearner.tick_graph) for 200+ ticks."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

N, CAP, BATCH = 4096, 1 << 20, 256


@pytest.fixture(scope="module")
def learner_mod():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from skillshot_learning_amd import learner
    return learner


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("exploration", ["action_noise", "param_noise"])
def test_config3_tick_graph(learner_mod, exploration, precision):
    """fp32 (the reference's precision, the learner's default) and the bf16
    opt-in, each in the tick form the learner picks by default"""
    L = learner_mod.SkillshotLearner(n_envs=N, device="cuda", seed=21, exploration=exploration, gamma=0.99,
                                     tau=0.005, replay_capacity=CAP, precision=precision)
    tg = L.tick_graph(batch=BATCH, ticks_per_graph=2, warmup=2)
    g = L.game_environment
    total0 = int(L.replay.total_t)
    adam0 = float(L.ddpg._fused.sa.steps[0])
    calls0 = int(L.ddpg.drop_calls)
    step0 = g.step_counter
    w0 = [p.clone() for p in L.model_actor.parameters()]
    g.clear_counters(stream=ctypes.c_void_p(tg.stream.cuda_stream))  # ordered after the capture's warm-up ticks (run() waits for the capture stream)
    tg.run(100)  # 200 ticks
    torch.cuda.synchronize()
    ticks = 200
    # ring: 2N transitions per tick, head / size from the device count
    assert int(L.replay.total_t) == total0 + ticks * 2 * N
    L.replay.sync_host()
    assert L.replay.size == min(L.replay.total, CAP) and L.replay.head == L.replay.total % CAP
    # engine RNG counter: one value per tick; Adam / dropout counters: one per update
    assert g.step_counter == step0 + ticks
    assert float(L.ddpg._fused.sa.steps[0]) == adam0 + ticks
    assert int(L.ddpg.drop_calls) == calls0 + ticks
    # actions the last tick took: tanh outputs (+ N(0, 0.15) with action noise)
    a = tg.act
    assert bool(torch.isfinite(a).all())
    if exploration == "param_noise":
        assert float(a.abs().max()) <= 1.0
    else:
        assert float(a.abs().max()) < 1.0 + 6 * 0.15
    for m in (L.model_actor, L.model_critic, L.ddpg.target_actor, L.ddpg.target_critic):
        assert all(bool(torch.isfinite(p).all()) for p in m.parameters())
    assert any((p - q).abs().max() > 0 for p, q in zip(L.model_actor.parameters(), w0))
    c = g.counters()
    assert c["dones"] > 0 and c["hits_p1"] + c["hits_p2"] <= c["dones"]
    # only episodes that ended inside the 200 counted ticks: each lasted <= 200 + the warm-up
    assert c["ticks_sum"] <= c["dones"] * (ticks + 8)
    # the replay rows hold finite observations in the reference's ranges
    rows = L.replay.buf[:min(L.replay.size, 65536)]
    assert bool(torch.isfinite(rows).all())
    assert bool(((rows[:, 2:4] >= 0) & (rows[:, 2:4] <= 1)).all())  # x / 250, y / 250 (:521-522)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_config3_fused_update_equals_autograd(learner_mod, precision):
    """one update of the config-3 learner on a sampled batch: the fused
    kernels' gradients against the torch autograd path at the same precision
    on the same batch and Dropout masks.  fp32 (the reference's precision):
    1e-4 relative Frobenius per parameter (measured ~1e-6: fp32 sums in
    another order; tests/test_learn32_gpu.py holds the kernels to 1e-5 of the
    fp64 Keras restatement).  bf16: 5 % (measured 0.2-2 % over seeds 22-24
    on the replay's real observations, tools/diag_config3.py; the rotation
    features reach ~9.9, so layer-1 operand rounding weighs more than on
    test_update_gpu's data)."""
    from test_update_gpu import _check_grads
    REL = 1e-4 if precision == "fp32" else 0.05
    L = learner_mod.SkillshotLearner(n_envs=N, device="cuda", seed=22, exploration="action_noise", gamma=0.99,
                                     tau=0.005, replay_capacity=CAP, precision=precision)
    L.train_ticks(4, batch=BATCH)
    s, a, r, s2, d = [t.clone() for t in L.replay.sample(BATCH)]
    fu = L.ddpg._fused
    c0 = fu.calls.clone()
    g = fu.grads("critic", s, a, s2=s2, r=r, d=d, gamma=0.99)
    # the autograd reference at the same precision (bf16: its bootstrap target
    # comes from the packed bf16 target nets, as the fused launch's does)
    ref = learner_mod.DDPG("cuda", seed=22, gamma=0.99, tau=0.005, fused_update=False, precision=precision)
    for dst, src in ((ref.model_actor, L.model_actor), (ref.model_critic, L.model_critic),
                     (ref.target_actor, L.ddpg.target_actor), (ref.target_critic, L.ddpg.target_critic)):
        dst.load_state_dict(src.state_dict())
    ref.drop_seed, ref.drop_calls = L.ddpg.drop_seed, c0.clone()
    with torch.no_grad():
        y = r + 0.99 * (1 - d) * ref.target_q(s2)
    ref.critic_step(s, a, y)
    _check_grads(g, ref.model_critic, [p.grad for p in ref.model_critic.parameters()], REL)
    ga = fu.grads("actor", s)
    # critic_step applied its Adam step to ref's critic; the fused grads()
    # launch does not update: the actor gradient is taken through the same
    # (pre-update) critic on both sides
    ref.model_critic.load_state_dict(L.model_critic.state_dict())
    ref.model_actor_fit_step(s)
    _check_grads(ga, ref.model_actor, [p.grad for p in ref.model_actor.parameters()], REL)
