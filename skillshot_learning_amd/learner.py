"""SkillshotLearner on PyTorch-ROCm over the batched GPU engine.

Mirrors SkillshotLearner.py (adrientremblay/Skillshot_Learning):
  * actor  12 -> 256 relu -> 128 relu -> 2 tanh, kernels N(0, 0.05), zero
    biases (model_define_actor, :70-96)
  * critic state -> 256 relu -> Dropout(0.2) -> concat(action) -> 128 relu
    -> 1 linear, glorot-uniform hidden kernels, N(0, 0.05) output kernel
    (model_define_critic, :98-121)
  * the reference update rule (models_fit :419-443, model_actor_fit_step
    :386-417): shuffle, critic MSE to the IMMEDIATE reward at batch 16 for one
    pass with dropout active, then per batch of 16 an actor step on
    -sum_batch Q(s, mu(s)) (critic in inference mode); Adam lr 1e-3, eps 1e-7
    (Keras defaults)
  * exploration (:215-281): deterministic, action noise N(0, 0.15), or
    parameter noise w <- w + w * N(0, 0.5) drawn afresh per player per tick.
    Batched, every (game, player) gets its own noisy actor; that is sampled
    EXACTLY in distribution by local reparameterisation (each noisy weight is
    used once per forward): per layer y = xW + b + 0.5 * sqrt(x^2 W^2 + b^2) * xi.

Build-side extensions (BASELINE.json north_star; no reference row): an HBM
replay ring (112 B per transition), target networks with soft update tau,
a discount gamma (0 keeps the reference's immediate-reward critic), and the
multi-GPU path: one process per GPU, games sharded by global id, gradients
all-reduced (RCCL over xGMI; gloo on CPU) as one flat bucket per update, and
each rank's sampled minibatch all-gathered into a shared batch.
"""
import ctypes
import math
import os
import warnings

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from ._capi import SkillshotError
from .rng import DROP_SCALE, dropout_keep

STATE_DIM = 12   # SkillshotLearner.py:54
ACTION_DIM = 2   # :55
MAX_DIST = (2 * (250 ** 2)) ** 0.5  # max_dist_normaliser, :43

# get_state() feature indices used by calculate_rewards (vec_env.FEATURE_KEYS)
_F_AGE, _F_DIST, _F_FC = 14, 16, 17


def calculate_rewards_full(dist, future_collision, age, winner, lengths=None, max_dist=MAX_DIST,
                           on_target_multiplier_reduction=0.25, loss_reward_multiplier=2,
                           base_reward_multiplier=0.75):
    """calculate_rewards (SkillshotLearner.py:605-661) batched over games.

    Inputs describe game_states[1:] of each game's episode, tick-major:
      dist [T, N, 2] float64   projectile_dist_opponent of players 1, 2
      future_collision [T, N, 2] bool   projectile_future_collision_opponent
      age [T, N, 2] int        projectile_age
      winner [T, N] int        game_winner (0, or the id the reference stores
                               in winner_id, SkillshotGame.py check_collision)
      lengths [N]              episode length per game (<= T; default T)
    Returns (rewards [T, N, 2] float64, raised [N] bool).

    Follows the reference statement by statement, quirks included:
      * per-player multiplier 0.75, 0.5 while the own projectile is on target
        (:632-635), 2.75 for the loser of a won tick (:637-639, overrides);
      * reward = (dist[opp] - dist[own] * multi + min_dist * 2) / max_dist
        with min_dist always 0: :643 reads game_state["projectile_cooldown"],
        a key the top-level state never has (SkillshotGame.py:139);
      * a won tick t sets rewards[t - age(winner)][winner] = 1 (:624-627),
        with Python list indexing over the t rewards built so far: a negative
        index wraps once, anything outside [-t, t) raises IndexError, which
        aborts the reference call; such games are flagged in `raised` and
        their rewards are NaN.
    """
    T, N = winner.shape
    dev = dist.device
    if lengths is None:
        lengths = torch.full((N,), T, dtype=torch.long, device=dev)
    lengths = lengths.to(dev).long()
    dist = dist.to(torch.float64)
    w = winner.long()
    base = torch.tensor(float(base_reward_multiplier), dtype=torch.float64, device=dev)
    multi = torch.where(future_collision.bool(), base - on_target_multiplier_reduction, base)
    loser = torch.where(w != 0, 3 - w, torch.zeros_like(w))  # the id in (1, 2) that is not winner_id
    pid = torch.arange(1, 3, device=dev).view(1, 1, 2)
    multi = torch.where(loser.unsqueeze(-1) == pid, base + loss_reward_multiplier, multi)
    r = (dist.flip(-1) - dist * multi) / max_dist
    tick = torch.arange(T, device=dev).view(T, 1)
    valid = tick < lengths.view(1, N)
    won = (w != 0) & valid
    raised = torch.zeros(N, dtype=torch.bool, device=dev)
    if bool(won.any()):
        t_idx, n_idx = torch.nonzero(won, as_tuple=True)
        wi = w[t_idx, n_idx] - 1
        f = t_idx - age.long()[t_idx, n_idx, wi]
        f = torch.where(f < 0, f + t_idx, f)             # list[-k] == list[len - k]
        bad = (f < 0) | (f >= t_idx)
        raised[n_idx[bad]] = True
        ok = ~bad
        r[f[ok], n_idx[ok], wi[ok]] = 1.0
    r = torch.where(valid.unsqueeze(-1), r, torch.full_like(r, float("nan")))
    r[:, raised] = float("nan")
    return r, raised


def _keras_normal_(t, std=0.05):
    with torch.no_grad():
        t.normal_(0.0, std)


def _glorot_uniform_(w):
    fan_out, fan_in = w.shape
    limit = math.sqrt(6.0 / (fan_in + fan_out))
    with torch.no_grad():
        w.uniform_(-limit, limit)


class Actor(nn.Module):
    """model_define_actor (SkillshotLearner.py:70-96)."""

    def __init__(self):
        super().__init__()
        self.l1 = nn.Linear(STATE_DIM, 256)
        self.l2 = nn.Linear(256, 128)
        self.l3 = nn.Linear(128, ACTION_DIM)
        for l in (self.l1, self.l2, self.l3):
            _keras_normal_(l.weight, 0.05)  # RandomNormal(0, 0.05), :74
            nn.init.zeros_(l.bias)          # Keras Dense default

    def forward(self, s):
        h = F.relu(self.l1(s))
        h = F.relu(self.l2(h))
        return torch.tanh(self.l3(h))

    def forward_param_noise(self, s, sd, generator=None):
        """Per-row independent parameter noise w' = w(1 + sd*eps), sampled by
        local reparameterisation (exact in distribution, see module doc)."""
        x = s
        for k, l in enumerate((self.l1, self.l2, self.l3)):
            mean = F.linear(x, l.weight, l.bias)
            var = F.linear(x * x, l.weight * l.weight, l.bias * l.bias)
            xi = torch.randn(mean.shape, device=mean.device, dtype=mean.dtype, generator=generator)
            y = mean + sd * torch.sqrt(var) * xi
            x = torch.tanh(y) if k == 2 else F.relu(y)
        return x


class Critic(nn.Module):
    """model_define_critic (SkillshotLearner.py:98-121)."""

    def __init__(self):
        super().__init__()
        self.l1 = nn.Linear(STATE_DIM, 256)
        self.drop = nn.Dropout(0.2)
        self.l2 = nn.Linear(256 + ACTION_DIM, 128)
        self.l3 = nn.Linear(128, 1)
        _glorot_uniform_(self.l1.weight)
        _glorot_uniform_(self.l2.weight)
        _keras_normal_(self.l3.weight, 0.05)  # kernel_initializer="RandomNormal"
        for l in (self.l1, self.l2, self.l3):
            nn.init.zeros_(l.bias)

    def forward(self, s, a, keep=None):
        """keep (bool [rows, 256], optional): the Dropout(0.2) keep-mask of a
        training step (rng.dropout_keep, the kernels' masks); without it
        nn.Dropout applies in train mode and nothing in eval mode."""
        h = F.relu(self.l1(s))
        h = h * (keep.to(h.dtype) * DROP_SCALE) if keep is not None else self.drop(h)
        h = F.relu(self.l2(torch.cat([h, a], dim=-1)))
        return self.l3(h)


class KerasAdam(torch.optim.Optimizer):
    """tf.keras.optimizers.Adam() of the reference (SkillshotLearner.py:68; the
    critic's compile("adam"), :118): lr 1e-3, beta_1 0.9, beta_2 0.999,
    epsilon 1e-7, and Keras' update rule (keras.optimizers.Adam.update_step,
    TensorFlow 2.x; the reference pins no version, and the older
    ResourceApplyAdam kernel is the same formula):

        m += (g - m) (1 - beta_1);   v += (g^2 - v) (1 - beta_2)
        alpha = lr sqrt(1 - beta_2^t) / (1 - beta_1^t)
        p -= m alpha / (sqrt(v) + epsilon)

    i.e. epsilon is added to sqrt(v) BEFORE the bias correction, where
    torch.optim.Adam adds it after.  Per-parameter state `exp_avg`,
    `exp_avg_sq` and `step` (a float32 tensor on the parameter's device, so a
    hipGraph capture replays it); k_adam_flat (csrc/sk_update.hip) computes
    the same formula."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-7):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))

    @torch.no_grad()
    def step(self, closure=None):
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                if st["step"].device != p.device or st["step"].dtype != torch.float32:  # e.g. after load_state_dict
                    st["step"] = st["step"].to(device=p.device, dtype=torch.float32)
                g, m, v = p.grad, st["exp_avg"], st["exp_avg_sq"]
                st["step"].add_(1.0)
                t = st["step"]
                m.add_((g - m) * (1.0 - b1))
                v.add_((g * g - v) * (1.0 - b2))
                alpha = group["lr"] * torch.sqrt(1.0 - torch.pow(b2, t)) / (1.0 - torch.pow(b1, t))
                p.sub_((m * alpha) / (torch.sqrt(v) + group["eps"]))
        return None


def keras_adam(params):
    """Keras Adam defaults (SkillshotLearner.py:68, :118)."""
    return KerasAdam(list(params), lr=1e-3, betas=(0.9, 0.999), eps=1e-7)


class ReplayRing:
    """Transitions (s 12f, a 2f, r 1f, s' 12f, done 1f = 112 B) in HBM, packed
    as one [capacity, 28] float32 row per transition (`s`, `a`, `r`, `s2`, `d`
    are column views).  `total` counts the rows ever inserted: head = total %
    capacity, size = min(total, capacity); the host keeps `total`, the device
    `total_t`.

    Two insert/sample paths: `add`/`sample` use the host count (slice copies,
    Python-int range); `add_dev`/`sample_dev` use the device count so a
    captured hipGraph inserts at the right row and samples the right range on
    every replay.  On the GPU those are one launch each (csrc/sk_replay.hip:
    `sk_replay_insert`, whose last workgroup advances `total_t`, and
    `sk_replay_sample`, a Philox gather into persistent contiguous batch
    buffers, which the next `sample_dev` of the same size overwrites)."""

    WIDTH = 2 * STATE_DIM + ACTION_DIM + 2

    def __init__(self, capacity, device, seed=0):
        self.cap = int(capacity)
        self.buf = torch.zeros(self.cap, self.WIDTH, device=device)
        self.s, self.a, self.r, self.s2, self.d = self._split(self.buf)
        self.total = 0
        self.total_t = torch.zeros((), dtype=torch.int64, device=device)
        self._ar = {}
        self.seed = int(seed) & ((1 << 64) - 1)
        self._k = None
        self._arrivals = None
        self._draws = 0
        self._batches = {}
        # the overlapped learner tick's sample counts: slot p holds the row
        # count before the insert of a tick of parity p (TickGraph)
        self.horizon = torch.zeros(2, dtype=torch.int64, device=device)
        if self.buf.is_cuda:
            from . import _capi
            self._k = _capi.load()
            self._arrivals = torch.zeros(288, dtype=torch.int32, device=device)  # SK_REPLAY_ARRIVAL_WORDS

    def arrivals(self):
        """the insert launches' arrival counters (SK_REPLAY_ARRIVAL_WORDS,
        left zeroed by every launch)"""
        if self._arrivals is None:
            self._arrivals = torch.zeros(288, dtype=torch.int32, device=self.buf.device)
        return self._arrivals

    head = property(lambda self: self.total % self.cap)
    size = property(lambda self: min(self.total, self.cap))
    head_t = property(lambda self: torch.remainder(self.total_t, self.cap))
    size_t = property(lambda self: torch.clamp(self.total_t, max=self.cap))

    @staticmethod
    def _split(rows):
        S, A = STATE_DIM, ACTION_DIM
        return (rows[:, :S], rows[:, S:S + A], rows[:, S + A], rows[:, S + A + 1:2 * S + A + 1],
                rows[:, 2 * S + A + 1])

    @staticmethod
    def _pack(s, a, r, s2, d):
        n = s.shape[0]
        if d.numel() != n:  # per-game done for player-major rows (row r -> game r % N)
            d = d.reshape(1, -1).expand(n // d.numel(), -1)
        # one kernel: cat promotes (e.g. a uint8 done column) to float32
        return torch.cat([s.reshape(n, STATE_DIM), a.reshape(n, ACTION_DIM), r.reshape(n, 1),
                          s2.reshape(n, STATE_DIM), d.reshape(n, 1)], 1).float()

    def add(self, s, a, r, s2, d):
        n = s.shape[0]
        rows = self._pack(s, a, r, s2, d)
        if n > self.cap:
            rows, n = rows[-self.cap:], self.cap
        head = self.head
        first = min(n, self.cap - head)  # contiguous copies, at most two
        self.buf[head:head + first].copy_(rows[:first])
        if first < n:
            self.buf[:n - first].copy_(rows[first:])
        self.total += n
        self.total_t.fill_(self.total)

    def sample(self, b, generator=None):
        idx = torch.randint(0, self.size, (b,), device=self.buf.device, generator=generator)
        return self._split(self.buf[idx])

    def add_dev(self, s, a, r, s2, d):
        """Capturable insert of n <= capacity rows at the device-side head; d is
        per row or per game (uint8 [n / 2] for the engine's [2, N] rows)."""
        n = s.shape[0]
        if n > self.cap:
            raise ValueError("add_dev: more rows than capacity")
        if self._k is not None:
            from . import _capi
            p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
            sc, ac = s.float().contiguous(), a.float().contiguous()
            rc, s2c = r.float().contiguous(), s2.float().contiguous()
            dc = d.contiguous() if d.dtype == torch.uint8 else (d != 0).to(torch.uint8).contiguous()
            _capi.check(self._k.sk_replay_insert(
                p(self.buf), self.cap, p(self.total_t), p(self._arrivals), p(sc), p(ac), p(rc), p(s2c), p(dc),
                dc.numel(), n, ctypes.c_void_p(torch.cuda.current_stream(self.buf.device).cuda_stream)))
        else:
            ar = self._ar.get(n)
            if ar is None:
                ar = self._ar[n] = torch.arange(n, dtype=torch.int64, device=self.buf.device)
            self.buf.index_copy_(0, torch.remainder(ar + self.total_t, self.cap), self._pack(s, a, r, s2, d))
            self.total_t.add_(n)
        self.total += n  # host mirror (exact while n is fixed)

    def add_sample_dev(self, s, a, r, s2, d, b):
        """add_dev followed by sample_dev(b) in one launch on the GPU
        (sk_replay_insert_sample, bit-identical to the two); the pair
        elsewhere."""
        if self._k is None:
            self.add_dev(s, a, r, s2, d)
            return self.sample_dev(b)
        from . import _capi
        n = s.shape[0]
        if n > self.cap:
            raise ValueError("add_sample_dev: more rows than capacity")
        out = self._batch_bufs(b)
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        sc, ac = s.float().contiguous(), a.float().contiguous()
        rc, s2c = r.float().contiguous(), s2.float().contiguous()
        dc = d.contiguous() if d.dtype == torch.uint8 else (d != 0).to(torch.uint8).contiguous()
        draw = self._draws
        self._draws = (self._draws + 1) & 0x7FFFFFFF
        _capi.check(self._k.sk_replay_insert_sample(
            p(self.buf), self.cap, p(self.total_t), p(self._arrivals), p(sc), p(ac), p(rc), p(s2c), p(dc),
            dc.numel(), n, self.seed, draw, b, *[p(t) for t in out],
            ctypes.c_void_p(torch.cuda.current_stream(self.buf.device).cuda_stream)))
        self.total += n
        return out

    def _batch_bufs(self, b):
        out = self._batches.get(b)
        if out is None:
            dev = self.buf.device
            out = self._batches[b] = (torch.empty(b, STATE_DIM, device=dev), torch.empty(b, ACTION_DIM, device=dev),
                                      torch.empty(b, device=dev), torch.empty(b, STATE_DIM, device=dev),
                                      torch.empty(b, device=dev))
        return out

    def next_draw(self, b):
        """(the batch buffers, the draw number) of the next device-side sample
        of b rows (sample_dev's, for a launch that gathers by itself)"""
        draw = self._draws
        self._draws = (self._draws + 1) & 0x7FFFFFFF
        return self._batch_bufs(b), draw

    def sample_dev(self, b, generator=None, exclude=0):
        """Capturable uniform sample over the device-side size (exclude > 0:
        over the min(count, cap - exclude) newest rows, sk_replay_sample_excl)."""
        if self._k is not None:
            from . import _capi
            out = self._batch_bufs(b)
            p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
            draw = self._draws
            self._draws = (self._draws + 1) & 0x7FFFFFFF
            _capi.check(self._k.sk_replay_sample_excl(
                p(self.buf), self.cap, p(self.total_t), self.seed, draw, b, *[p(t) for t in out], int(exclude),
                ctypes.c_void_p(torch.cuda.current_stream(self.buf.device).cuda_stream)))
            return out
        if exclude:
            raise ValueError("exclude needs the device ring")
        u = torch.rand(b, dtype=torch.float64, device=self.buf.device, generator=generator)
        size_t = self.size_t
        idx = torch.minimum((u * size_t).long(), size_t - 1)
        return self._split(self.buf[idx])

    def sync_host(self):
        self.total = int(self.total_t)


class DDPG:
    """Actor/critic, optimisers and update rules (device-agnostic: CPU tests
    and gloo multi-process tests drive it without a GPU).

    Dropout of a critic training step is keyed by (dropout seed, call number,
    GLOBAL batch row, unit) on every path (rng.dropout_keep on the torch path,
    the same Philox draw inside k_critic_grad), and every loss is normalised by
    the global batch, so an update split over ranks equals, up to fp32
    summation order, the 1-rank update on the concatenated batch.

    Multi-rank (one process per GPU, games sharded by global id; the seed is
    shared, rank_seed_offset separates the ranks' replay draws):
      multi_rank="grad"    (BASELINE config 4) every rank samples `batch` rows
                           of its own replay ring, computes the gradient of its
                           rows (global rows rank*batch ..), and the gradients
                           are summed by one all-reduce per net;
      multi_rank="shared"  (config 5, shared replay) the ranks' samples are
                           all-gathered into one [world*batch] batch and rank r
                           takes the strided slice r::world of it (rows of
                           every rank), global rows rank*batch .., then the
                           same gradient all-reduce.
    Per-rank update work is `batch` rows whatever the world size."""

    def __init__(self, device="cpu", seed=0, batch_size=16, gamma=0.0, tau=None, replay_capacity=0,
                 process_group=None, rank_seed_offset=0, fused_update=None, multi_rank="grad", precision="fp32",
                 force_collectives=False):
        self.device = torch.device(device)
        torch.manual_seed(seed)
        self.model_actor = Actor().to(self.device)
        self.model_critic = Critic().to(self.device)
        self.group = process_group
        # run the multi-rank update (collectives and all) even on a 1-rank
        # group: a one-GPU rehearsal of the RCCL path that configs 4 and 5
        # take (tests/test_rccl_capture_gpu.py)
        self.force_collectives = bool(force_collectives)
        if multi_rank not in ("grad", "shared"):
            raise ValueError("multi_rank must be 'grad' or 'shared'")
        self.multi_rank = multi_rank
        self.precision = precision
        self._sync_params()
        self.optimiser = keras_adam(self.model_actor.parameters())         # SkillshotLearner.py:68
        self.critic_optimiser = keras_adam(self.model_critic.parameters())  # critic.compile("adam"), :118
        self.model_param_batch_size = batch_size
        self.gamma = float(gamma)
        self.tau = tau
        if tau is not None:
            self.target_actor = Actor().to(self.device)
            self.target_critic = Critic().to(self.device)
            self.target_actor.load_state_dict(self.model_actor.state_dict())
            self.target_critic.load_state_dict(self.model_critic.state_dict())
        self.replay = (ReplayRing(replay_capacity, self.device, seed=seed * 7919 + rank_seed_offset + 29)
                       if replay_capacity else None)
        self._tq = None  # fused target-Q kernel (GPU), created at first use
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed * 7919 + rank_seed_offset + 17)
        # Dropout key: the same on every rank (masks are keyed by global row);
        # the call number lives on device (advanced once per critic step)
        self.drop_seed = (seed * 1000033 + 5) & ((1 << 64) - 1)
        self.drop_calls = torch.zeros(1, dtype=torch.int64, device=self.device)
        # the update on MFMA kernels (update_kernel.FusedUpdate) on the GPU;
        # SK_FUSED_UPDATE=0 / fused_update=False keeps the autograd path
        if fused_update is None:
            fused_update = self.device.type == "cuda" and os.environ.get("SK_FUSED_UPDATE", "1") != "0"
        self._fused = None
        if fused_update:
            from .update_kernel import FusedUpdate
            self._fused = FusedUpdate(self)

    # ------------------------------------------------------------ distributed
    def world(self):
        return dist.get_world_size(self.group) if dist.is_available() and dist.is_initialized() else 1

    def rank(self):
        return dist.get_rank(self.group) if self.world() > 1 else 0

    def multi(self):
        """the update goes through the collectives (more than one rank, or a
        forced 1-rank rehearsal)"""
        return self.world() > 1 or (self.force_collectives and dist.is_available() and dist.is_initialized())

    def _sync_params(self):
        """Start every rank from rank 0's weights (broadcast)."""
        if self.world() > 1:
            for m in (self.model_actor, self.model_critic):
                for p in m.parameters():
                    dist.broadcast(p.data, src=0, group=self.group)

    # every collective of an update goes through _collective: eager it runs
    # at once; while a TickGraph captures in segments it cuts the capture
    # there and is replayed between the graph segments (collective_hook)
    collective_hook = None

    def _collective(self, fn):
        if self.collective_hook is not None:
            self.collective_hook(fn)
        else:
            fn()

    def allreduce_sum(self, flat):
        """in-place SUM all-reduce of one flat device buffer (RCCL over xGMI)"""
        self._collective(lambda: dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group))

    def _allreduce_grads(self, module):
        """Gradient all-reduce (sum: each rank's loss is already normalised
        by the global batch) as ONE flat bucket per update: 36,482 actor /
        36,609 critic fp32 parameters (RCCL over xGMI)."""
        if not self.multi():
            return
        grads = [p.grad for p in module.parameters()]
        flat = torch.cat([g.reshape(-1) for g in grads])
        self.allreduce_sum(flat)
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n

    def _allgather_batch(self, *tensors):
        """Shared replay sample: every rank contributes its local minibatch,
        one all-gather of a packed buffer; returns the [world*b] batch (rank
        0's rows first)."""
        w = self.world()
        if not self.multi():
            return tensors
        flat = torch.cat([t.reshape(t.shape[0], -1) for t in tensors], dim=1).contiguous()
        out = torch.empty((w * flat.shape[0], flat.shape[1]), device=flat.device, dtype=flat.dtype)
        if flat.is_cuda and dist.get_backend(self.group) == "gloo":  # gloo: the list form on device tensors
            self._collective(lambda: dist.all_gather(list(out.chunk(w)), flat, group=self.group))
        else:
            self._collective(lambda: dist.all_gather_into_tensor(out, flat, group=self.group))
        res, off = [], 0
        for t in tensors:
            k = t[0].numel()
            res.append(out[:, off:off + k].reshape((out.shape[0],) + tuple(t.shape[1:])))
            off += k
        return tuple(res)

    # ------------------------------------------------------------ updates
    def critic_step(self, s, a, target, row_offset=0, global_batch=None):
        """One critic Adam step on MSE(Q(s, a), target) with Dropout active
        (critic.fit, SkillshotLearner.py:434): loss = sum over this rank's
        rows of (Q - y)^2 / global_batch (= the batch mean on one rank)."""
        B = s.shape[0]
        gb = B if global_batch is None else int(global_batch)
        if self._fused is not None:  # one MFMA gradient launch + one Adam launch
            return self._fused.critic_step(s, a, target, row_offset=row_offset, global_batch=gb)
        self.model_critic.train()
        keep = dropout_keep(self.drop_seed, self.drop_calls, row_offset, B, device=s.device)
        q = self.model_critic(s, a, keep=keep).squeeze(-1)
        loss = ((q - target) ** 2).sum() / gb
        self.critic_optimiser.zero_grad(set_to_none=True)  # backward writes the grads (no accumulate)
        loss.backward()
        self.drop_calls.add_(1)
        self._allreduce_grads(self.model_critic)
        self.critic_optimiser.step()
        return loss.detach()

    def model_actor_fit_step(self, s):
        """model_actor_fit_step (:386-417): actor grads with output_gradients =
        -dQ/da, i.e. descent on -sum_batch Q(s, mu(s)); critic in inference
        mode.  Multi-rank: each rank's -sum over its rows, gradients summed."""
        if self._fused is not None:
            return self._fused.actor_step(s)
        self.model_critic.eval()
        for p in self.model_critic.parameters():
            p.requires_grad_(False)
        q = self.model_critic(s, self.model_actor(s))
        loss = -q.sum()
        self.optimiser.zero_grad(set_to_none=True)
        loss.backward()
        for p in self.model_critic.parameters():
            p.requires_grad_(True)
        self._allreduce_grads(self.model_actor)
        self.optimiser.step()
        return loss.detach()

    def models_fit(self, states, actions, rewards):
        """models_fit (:419-443): shuffle, critic one pass at batch 16, then the
        actor per batch of 16 on the same shuffled states.  No target nets
        or soft update here (the reference has none)."""
        assert states.shape[0] == actions.shape[0] == rewards.shape[0]
        idx = torch.randperm(states.shape[0], device=states.device, generator=self.gen)
        states, actions, rewards = states[idx], actions[idx], rewards[idx]
        b = self.model_param_batch_size
        n = states.shape[0]
        fu = self._fused
        if fu is not None:
            fu.soft_update_in_adam = False
        # the resident passes (csrc/sk_fit.hip; fp32, one rank, batch 16):
        # every full minibatch of a pass in launches that hold the net on
        # chip; SK_FIT_RESIDENT=0 keeps the three-launch steps
        resident = (fu is not None and fu.f32 and states.is_cuda and not self.multi() and b == fu.FIT_ROWS and
                    os.environ.get("SK_FIT_RESIDENT", "1") != "0")
        if resident:
            try:
                done = self._resident_pass(fu, True, lambda: fu.fit_critic(states, actions, rewards)) * b
                for k in range(done, n, b):  # the partial last minibatch (or the whole pass, after a failure)
                    self.critic_step(states[k:k + b], actions[k:k + b], rewards[k:k + b])
                self._actor_pass(states, b, n)
            finally:
                fu.soft_update_in_adam = True
            return
        # graph-replayed chunks of FIT_CHUNK minibatches (the fused kernels,
        # one rank): the same launches on the same rows, staged into fixed
        # buffers, without ~0.1 ms of host time per minibatch; the first
        # minibatch of each pass runs eagerly (it warms the launch path the
        # capture records) and the remainder after the last whole chunk too
        graph = (fu is not None and states.is_cuda and not self.multi() and n >= 2 * b and
                 os.environ.get("SK_FIT_GRAPH", "1") != "0")
        M = self.FIT_CHUNK
        chunks = (n // b - 1) // M if graph else 0
        try:
            for k in range(0, n, b):
                if chunks and k == b:
                    self._fit_chunks(states, actions, rewards, b, M, chunks, critic=True)
                if chunks and b <= k < b + chunks * M * b:
                    continue
                self.critic_step(states[k:k + b], actions[k:k + b], rewards[k:k + b])
            for k in range(0, n, b):
                if chunks and k == b:
                    self._fit_chunks(states, actions, rewards, b, M, chunks, critic=False)
                if chunks and b <= k < b + chunks * M * b:
                    continue
                self.model_actor_fit_step(states[k:k + b])
        finally:
            if fu is not None:
                fu.soft_update_in_adam = True

    @staticmethod
    def _resident_pass(fu, critic, run):
        """one resident models_fit pass, checked before the next pass reads
        its net (one host sync per pass).  A launch the device refuses
        (SK_EHIP: its LDS limit or the attribute call, before anything ran)
        or an in-launch exchange lost (fit_check) restores the net as it was
        and returns 0 minibatches done: the caller runs the whole pass on the
        three-launch steps"""
        snap = fu.fit_snapshot(critic)
        try:
            done = run()
            fu.fit_check()
            return done
        except SkillshotError as e:
            fu.fit_restore(snap)
            warnings.warn(f"resident models_fit pass failed ({e}); rerunning it on the three-launch steps")
            return 0

    def _actor_pass(self, states, b, n):
        """models_fit's actor pass (:436-443) on the fused kernels: resident
        launches (sk_fit_actor_f32) for every full minibatch and the partial
        last one eager; SK_FIT_RESIDENT=critic keeps the three-launch steps
        for this pass (the first minibatch eager, captured chunks of
        FIT_CHUNK, the rest eager)"""
        if os.environ.get("SK_FIT_RESIDENT", "1") != "critic":
            fu = self._fused
            done = self._resident_pass(fu, False, lambda: fu.fit_actor(states)) * b
            for k in range(done, n, b):
                self.model_actor_fit_step(states[k:k + b])
            return
        graph = self._fused is not None and states.is_cuda and not self.multi() and n >= 2 * b and \
            os.environ.get("SK_FIT_GRAPH", "1") != "0"
        M = self.FIT_CHUNK
        chunks = (n // b - 1) // M if graph else 0
        for k in range(0, n, b):
            if chunks and k == b:
                self._fit_chunks(states, None, None, b, M, chunks, critic=False)
            if chunks and b <= k < b + chunks * M * b:
                continue
            self.model_actor_fit_step(states[k:k + b])

    FIT_CHUNK = 64  # minibatches per captured models_fit graph

    def _fit_chunks(self, states, actions, rewards, b, M, chunks, critic):
        """rows [b, b + chunks M b) of one models_fit pass as `chunks` replays
        of a captured graph of M critic (or actor) steps on staging buffers"""
        key = (b, M, bool(critic))
        cache = self.__dict__.setdefault("_fit_graphs", {})
        if key not in cache:
            dev = states.device
            S = torch.empty((M * b, STATE_DIM), dtype=torch.float32, device=dev)
            A = torch.empty((M * b, ACTION_DIM), dtype=torch.float32, device=dev)
            R = torch.empty(M * b, dtype=torch.float32, device=dev)
            g = torch.cuda.CUDAGraph()
            torch.cuda.current_stream(dev).synchronize()
            # the captured steps' losses go to slots of their own (every
            # replay rewrites them), not to the eager steps' history
            with self._fused.private_loss_slots(M) as losses:
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    for m in range(M):
                        sl = slice(m * b, (m + 1) * b)
                        if critic:
                            self.critic_step(S[sl], A[sl], R[sl])
                        else:
                            self.model_actor_fit_step(S[sl])
            cache[key] = (g, S, A, R, losses)
        g, S, A, R, _ = cache[key]
        for j in range(chunks):
            lo = b + j * M * b
            S.copy_(states[lo:lo + M * b])
            if critic:
                A.copy_(actions[lo:lo + M * b])
                R.copy_(rewards[lo:lo + M * b])
            g.replay()

    def sample_local(self, batch, device_sampling=False):
        """this rank's minibatch of the replay ring"""
        if device_sampling:
            return self.replay.sample_dev(batch, generator=self.gen)
        return self.replay.sample(batch, generator=self.gen)

    def replay_update(self, batch, device_sampling=False):
        """Build-side extension: one critic + one actor step on a replay
        minibatch (see the class doc for the multi-rank schemes), optional
        bootstrapped target with target nets and soft update tau.
        device_sampling draws the minibatch over the ring's device-side size
        (hipGraph capture)."""
        return self.update_batch(*self.sample_local(batch, device_sampling))

    def update_overlapped(self, batch, total, exclude, before_actor_adam=None, step_job=None, job_in="critic"):
        """The overlapped tick's update (TickGraph, SK_TICK_OVERLAP): the
        critic step and the actor gradient on a minibatch keyed on `total`
        (the count before this tick's insert) that leaves out the `exclude`
        rows the insert running beside it writes, then before_actor_adam()
        (the join with the acting stream), then the actor's Adam launch.
        step_job: the tick's prepared acting launch, run in the critic's
        (job_in "critic") or the actor's ("actor") gradient backward launch
        (the fused overlapped tick)."""
        fu = self._fused
        w, rk, b = self.world(), self.rank(), int(batch)
        if w > 1 and b % 4:
            raise ValueError("multi-rank batches must be a multiple of 4 rows (Dropout key groups)")
        if self.multi() and self.multi_rank == "shared":
            # the shared replay: this rank's rows drawn as at `total` (the
            # stream-ordered count: the acting launch runs after this), the
            # ranks' rows all-gathered, the strided slice rk::w stepped
            s, a, r, s2, d = self.replay.sample_dev(b, exclude=exclude)
            s, a, r, s2, d = [t[rk::w] for t in self._allgather_batch(s, a, r, s2, d)]
            cj = step_job if job_in == "critic" else None
            if self.gamma > 0.0:
                lc = fu.critic_step(s, a, s2=s2, r=r, d=d, gamma=self.gamma, row_offset=rk * b, global_batch=w * b,
                                    step_job=cj)
            else:
                lc = fu.critic_step(s, a, r, row_offset=rk * b, global_batch=w * b, step_job=cj)
            return lc, fu.actor_step(s, before_adam=before_actor_adam, step_job=None if cj is not None else step_job)
        cj = step_job if job_in == "critic" else None
        lc, (s, _, _, _, _) = fu.critic_step_sampled(self.replay, b, gamma=self.gamma, row_offset=rk * b,
                                                     global_batch=w * b, total=total, exclude=exclude, step_job=cj)
        return lc, fu.actor_step(s, before_adam=before_actor_adam, step_job=None if cj is not None else step_job)

    def update_sampled(self, batch):
        """replay_update(batch, device_sampling=True) with the minibatch drawn
        inside the critic step's (first) launch where the kernels do that (the
        fused path at either precision, one rank or multi_rank "grad"): one
        launch fewer per update, bit-identical (the same Philox rows as
        sample_dev)."""
        fu = self._fused
        if fu is None or (self.multi() and self.multi_rank == "shared"):
            return self.replay_update(batch, device_sampling=True)
        w, rk, b = self.world(), self.rank(), int(batch)
        if w > 1 and b % 4:
            raise ValueError("multi-rank batches must be a multiple of 4 rows (Dropout key groups)")
        lc, (s, _, _, _, _) = fu.critic_step_sampled(self.replay, b, gamma=self.gamma, row_offset=rk * b,
                                                     global_batch=w * b)
        return lc, fu.actor_step(s)

    def update_batch(self, s, a, r, s2, d):
        """replay_update on this rank's sampled rows s, a, r, s2, d."""
        w, rk, b = self.world(), self.rank(), s.shape[0]
        if self.multi() and self.multi_rank == "shared":
            s, a, r, s2, d = [t[rk::w] for t in self._allgather_batch(s, a, r, s2, d)]
        row0, gb = rk * b, w * b
        if w > 1 and b % 4:
            raise ValueError("multi-rank batches must be a multiple of 4 rows (Dropout key groups)")
        if self._fused is not None:  # critic step (bootstrap inside) + actor step: 4 launches, Adam writes packs
            if self.gamma > 0.0:
                lc = self._fused.critic_step(s, a, s2=s2, r=r, d=d, gamma=self.gamma, row_offset=row0,
                                             global_batch=gb)
            else:
                lc = self._fused.critic_step(s, a, r, row_offset=row0, global_batch=gb)
            return lc, self._fused.actor_step(s)
        target = r
        if self.gamma > 0.0:
            with torch.no_grad():
                if self.device.type == "cuda" and self.precision == "bf16":  # r + gamma (1 - d) Q' in one launch
                    target = self._target_kernel().target(s2, r, d, self.gamma)
                else:
                    target = r + self.gamma * (1.0 - d) * self.target_q(s2)
        lc = self.critic_step(s, a, target, row_offset=row0, global_batch=gb)
        la = self.model_actor_fit_step(s)
        if self.tau is not None:
            self.soft_update()
        return lc, la

    @torch.no_grad()
    def target_q(self, s2):
        """Q'(s', mu'(s')) with the target nets (the online nets when tau is
        None).  On the GPU (bf16 kernels) one fused MFMA launch (sk_target_q)
        on weights packed after every change of the nets; otherwise the torch
        modules."""
        actor_t = self.target_actor if self.tau is not None else self.model_actor
        critic_t = self.target_critic if self.tau is not None else self.model_critic
        if self.device.type != "cuda" or self.precision != "bf16":
            critic_t.eval()
            return critic_t(s2, actor_t(s2)).squeeze(-1)
        return self._target_kernel()(s2)

    def _target_kernel(self):
        """The fused target kernel (critic_kernel.TargetQKernel) on packs that
        are current for the nets it reads."""
        if self._tq is None:
            from .critic_kernel import TargetQKernel
            actor_t = self.target_actor if self.tau is not None else self.model_actor
            critic_t = self.target_critic if self.tau is not None else self.model_critic
            self._tq = TargetQKernel(actor_t, critic_t)
        elif self.tau is None or self._fused is not None:
            self._tq.refresh()  # the nets it reads moved since the last call
        return self._tq

    @torch.no_grad()
    def soft_update(self):
        """target <- target + tau (online - target), one multi-tensor op per net."""
        for tgt, src in ((self.target_actor, self.model_actor), (self.target_critic, self.model_critic)):
            torch._foreach_lerp_(list(tgt.parameters()), list(src.parameters()), self.tau)
        if self._tq is not None:
            self._tq.refresh()

    def optimisers_loaded(self):
        """after Optimizer.load_state_dict replaced the Adam state tensors:
        the fused path copies them into its flat buffers and rebinds the views"""
        if self._fused is not None:
            self._fused.rebind_optimisers()


class SkillshotLearner:
    """Batched self-play DDPG learner (SkillshotLearner.py:13-682 API shape).

    n_envs games on `device` (global ids env_offset.. when sharded over
    ranks); both players of every game are driven by the same actor (self-play,
    :304-308).
    """
    player_ids = (1, 2)

    def __init__(self, n_envs=1, device="cuda", seed=0, env_offset=0, exploration="param_noise",
                 tick_limit=2000, use_random_start=True, replay_capacity=1 << 20, batch_size=16,
                 gamma=0.0, tau=None, actor_kernel=True, process_group=None, precision="fp32",
                 multi_rank="grad", force_collectives=False):
        from .vec_env import VecSkillshotGame
        if precision not in ("bf16", "fp32"):
            raise ValueError("precision must be 'bf16' or 'fp32'")
        self.precision = precision
        self.device = torch.device(device)
        self.game_environment = VecSkillshotGame(n_envs, device=self.device, seed=seed, env_offset=env_offset,
                                                 tick_limit=tick_limit, random_positions=use_random_start)
        self.n_envs = n_envs
        # every game starts its first episode the way model_train starts each
        # epoch, game_reset(random_positions=use_random_start) (:291); auto-
        # reset then keeps that start mode for later episodes
        self.game_environment.reset(random_positions=use_random_start)
        self.max_dist_normaliser = MAX_DIST                    # :43
        self.use_random_start = use_random_start               # :44
        self.dim_state_space, self.dim_action_space, self.dim_reward_space = STATE_DIM, ACTION_DIM, 1
        self.model_param_game_tick_limit = tick_limit          # :62
        self.action_noise_sd = 0.15                            # :63
        self.param_noise_sd = 0.5                              # :64
        self.exploration = exploration
        # on-disk locations (:46-51; formats in persist.py)
        self.save_location = "training_models"
        self.actor_dir_name, self.critic_dir_name = "actor", "critic"
        self.training_progress_dir_name, self.training_boards_dir_name = "training_progress", "training_boards"
        self.ddpg = DDPG(self.device, seed=seed, batch_size=batch_size, gamma=gamma, tau=tau,
                         replay_capacity=replay_capacity, process_group=process_group, rank_seed_offset=env_offset,
                         multi_rank=multi_rank, precision=precision, force_collectives=force_collectives)
        self.gen = self.ddpg.gen
        self.actor_kernel = None
        if actor_kernel and self.device.type == "cuda":
            from .actor_kernel import ActorKernel, ActorKernel32
            if precision == "fp32":  # flat fp32 parameters + the split pack the actor's Adam launch rewrites
                self.actor_kernel = ActorKernel32(self.model_actor, seed=seed * 1000003 + env_offset)
                if self.ddpg._fused is not None:
                    self.ddpg._fused.split_pack = self.actor_kernel.pack
            else:
                self.actor_kernel = ActorKernel(self.model_actor, seed=seed * 1000003 + env_offset)
                if self.ddpg._fused is not None:  # the actor's Adam launch writes the forward pack too
                    self.ddpg._fused.fwd_pack = self.actor_kernel.buf
        self.progress = dict(epoch_ticks=[], epoch_winner=[])

    # reference attribute names
    model_actor = property(lambda self: self.ddpg.model_actor)
    model_critic = property(lambda self: self.ddpg.model_critic)
    optimiser = property(lambda self: self.ddpg.optimiser)
    replay = property(lambda self: self.ddpg.replay)
    model_param_batch_size = property(lambda self: self.ddpg.model_param_batch_size)

    def models_fit(self, states, actions, rewards):
        self.ddpg.models_fit(states, actions, rewards)
        self._refresh_actor_pack()

    def _refresh_actor_pack(self):
        """repack the actor forward kernel's weights after an update, unless
        the fused update's Adam launch already wrote them"""
        if self.actor_kernel is None:
            return
        fu = self.ddpg._fused
        if fu is not None and self.actor_kernel.buf is not None and fu.fwd_pack is self.actor_kernel.buf:
            return
        if fu is not None and getattr(self.actor_kernel, "pack", None) is not None and \
                fu.split_pack is self.actor_kernel.pack:
            return
        self.actor_kernel.refresh()

    def replay_update(self, batch):
        return self.ddpg.replay_update(batch)

    # ------------------------------------------------------------ acting
    def prepare_states(self):
        """prepare_states (:512-543) of the current state: obs [2, N, 12]."""
        obs, _ = self.game_environment.observe()
        return obs

    @torch.no_grad()
    def model_act(self, obs, mode=None):
        """Actions [2, N, 2] for obs [2, N, 12] (model_act* :215-281)."""
        mode = mode or self.exploration
        x = obs.reshape(-1, STATE_DIM)
        if mode == "param_noise":
            if self.actor_kernel is not None:
                a = self.actor_kernel(x, noise_sd=self.param_noise_sd, generator=self.gen)
            else:
                a = self.model_actor.forward_param_noise(x, self.param_noise_sd, generator=self.gen)
        elif mode == "action_noise" and getattr(self.actor_kernel, "fused_action_noise", False):
            a = self.actor_kernel(x, action_sd=self.action_noise_sd)
        else:
            a = self.actor_kernel(x) if self.actor_kernel is not None else self.model_actor(x)
            if mode == "action_noise":
                a = a + self.action_noise_sd * torch.randn(a.shape, device=a.device, generator=self.gen)
        return a.reshape(2, -1, ACTION_DIM).contiguous()

    def do_actions(self, actions, reset_obs=True):
        """do_actions for both players + game_tick + obs/reward (:206-213, :312-324)."""
        return self.game_environment.step(actions, obs=True, reward="looking", auto_reset=True,
                                          reset_obs=reset_obs)

    # ------------------------------------------------------------ training loops
    def model_train(self, epochs, save_progress=False, save_boards=False, reward="looking", board_game=0):
        """model_train (:283-384) with the reference update rule: each epoch
        resets every game (random start), plays until every game has ended
        (hit or tick limit), then fits on all of the epoch's transitions of both
        players.  reward picks the reference's reward function for the epoch
        (:324-326): "looking" (the one it uses), "simple", or "full"
        (calculate_rewards, computed once the episode is complete; a game on
        which the reference would raise IndexError contributes no
        transitions).  save_progress writes the models and the epochs' ticks /
        winners, save_boards the board sequence of game `board_game` for
        every epoch (:370-384; formats in persist.py)."""
        g = self.game_environment
        full = reward == "full"
        call = dict(epoch_ticks=[], epoch_winner=[], epoch_board_sequences=[])
        # the episodes on device in one launch (sk_env_act_episode) where the
        # fp32 acting kernel runs them; the per-tick loop below otherwise
        # (bf16 / torch actors, the full reward's per-tick features, boards)
        on_device = (not full and not save_boards and self.actor_kernel is not None and
                     getattr(self.actor_kernel, "fused_act_step", False) and self.n_envs % 4 == 0 and
                     os.environ.get("SK_EPISODE_KERNEL", "1") != "0")
        for _ in range(epochs):
            g.reset(random_positions=self.use_random_start)
            obs = self.prepare_states()
            if on_device:
                ticks, winner = self._episode_on_device(obs, reward)
                for d in (self.progress, call):
                    d["epoch_ticks"].append(ticks.cpu())
                    d["epoch_winner"].append(winner.cpu())
                continue
            alive = torch.ones(self.n_envs, dtype=torch.bool, device=self.device)
            S, A, R, K, FT, W = [], [], [], [], [], []
            ticks = torch.zeros(self.n_envs, dtype=torch.int32, device=self.device)
            lengths = torch.zeros(self.n_envs, dtype=torch.long, device=self.device)
            winner = torch.zeros(self.n_envs, dtype=torch.uint8, device=self.device)
            boards = []
            while bool(alive.any()):
                act = self.model_act(obs)
                out = g.step(act, obs=True, reward="looking" if full else reward, auto_reset=False)
                keep = alive.repeat(2)
                S.append(obs.reshape(-1, STATE_DIM))
                A.append(act.reshape(-1, ACTION_DIM))
                K.append(keep)
                if full:
                    f = g.features()
                    FT.append(f[..., [_F_DIST, _F_FC, _F_AGE]])
                    W.append(out["winner"].long())
                else:
                    R.append(out["reward"].reshape(-1))
                done = out["done"].bool()
                newly = alive & done
                ticks = torch.where(newly, g.ticks, ticks)
                winner = torch.where(newly, out["winner"], winner)
                lengths = lengths + alive.long()
                if save_boards and bool(alive[board_game]):  # the board after each tick (:315-317)
                    boards.append(g.get_board(board_game).astype(np.int8))
                alive = alive & ~done
                obs = out["obs"]
            if full:
                ft = torch.stack(FT)                              # [T, N, 2, 3]
                rf, raised = calculate_rewards_full(ft[..., 0], ft[..., 1] != 0, ft[..., 2].long(),
                                                    torch.stack(W), lengths, self.max_dist_normaliser)
                R = [rt.t().reshape(-1).float() for rt in rf]    # [2N] player-major per tick
                K = [k & ~raised.repeat(2) for k in K]
            K = torch.cat(K)
            self.models_fit(torch.cat(S)[K], torch.cat(A)[K], torch.cat(R)[K])
            for d in (self.progress, call):
                d["epoch_ticks"].append(ticks.cpu())
                d["epoch_winner"].append(winner.cpu())
            if save_boards:
                call["epoch_board_sequences"].append(np.stack(boards) if boards else
                                                     np.zeros((0, 250, 250), np.int8))
        if save_progress:
            self.save_actor_critic_models(epochs)
            self.save_training_progress(call)
        if save_boards:
            self.save_training_boards(call["epoch_board_sequences"])
        return self.progress

    def _episode_on_device(self, obs, reward):
        """one model_train epoch with the episodes collected in one launch
        (VecSkillshotGame.act_episode: every game until it ends, the actor
        fixed, fresh noise per tick), then models_fit on the played rows in
        the per-tick loop's order (tick, player, game).  Returns the games'
        final ticks and winners."""
        g = self.game_environment
        mode = self.exploration
        kw = dict(noise_sd=self.param_noise_sd if mode == "param_noise" else 0.0,
                  action_sd=self.action_noise_sd if mode == "action_noise" else 0.0, reward=reward)
        # chunks of C ticks: the launch's buffers hold C + 1
        # state slabs (120 B per game-tick with actions and rewards), so a
        # large batch does not allocate tick_limit of them up front; each
        # chunk's played rows are compacted, in the loop's (tick, player,
        # game) order, and a chunk that ends short of C ends the episode
        C = self.episode_chunk_ticks()
        S, A, R = [], [], []
        while True:
            ep = g.act_episode(self.actor_kernel, obs, n_ticks=C, out=getattr(self, "_episode_bufs", None), **kw)
            self._episode_bufs = ep
            lengths = ep["lengths"].long()
            T = int(lengths.max()) if self.n_envs else 0
            keep = (torch.arange(T, device=self.device)[:, None] < lengths[None, :])[:, None, :].expand(
                T, 2, self.n_envs)
            S.append(ep["states"][:T][keep])
            A.append(ep["actions"][:T][keep])
            R.append(ep["rewards"][:T][keep])
            if T < C:
                break
            obs = ep["states"][C]
        self.models_fit(torch.cat(S), torch.cat(A), torch.cat(R))
        return g.ticks.clone(), g.winner_id.clone()

    def episode_chunk_ticks(self, share=0.125):
        """ticks per episode launch: the tick limit, or fewer where the
        launch's buffers (120 B per game-tick) would pass `share` of the
        device's free memory; SK_EPISODE_CHUNK overrides"""
        env = os.environ.get("SK_EPISODE_CHUNK")
        if env:
            return max(1, int(env))
        free, _ = torch.cuda.mem_get_info(self.device)
        per_tick = 120 * max(1, self.n_envs)
        return int(max(1, min(self.game_environment.tick_limit, (share * free) // per_tick)))

    # ------------------------------------------------------------ on-disk formats (persist.py)
    def save_actor_critic_models(self, epochs):
        from . import persist
        return persist.save_actor_critic_models(self.save_location, self.model_actor, self.model_critic, epochs)

    def load_actor_critic_models(self, load_index=-1):
        from . import persist
        ok = persist.load_actor_critic_models(self.save_location, self.model_actor, self.model_critic, load_index)
        if ok:
            self._params_changed()
        return ok

    def save_training_progress(self, total_progress):
        from . import persist
        return persist.save_training_progress(self.save_location, total_progress)

    def load_training_progress(self):
        from . import persist
        return persist.load_training_progress(self.save_location)

    def save_training_boards(self, epoch_board_list):
        from . import persist
        return persist.save_training_boards(self.save_location, epoch_board_list)

    def load_training_boards(self):
        from . import persist
        return persist.load_training_boards(self.save_location)

    def train_ticks(self, n_ticks, batch=256, updates_per_tick=1, warmup=None):
        """Build-side replay training: each tick acts
        with the exploration policy for every game, steps (auto-reset), pushes
        2N transitions into the HBM ring and runs `updates_per_tick` critic +
        actor updates on `batch`-sized samples."""
        g = self.game_environment
        obs = self.prepare_states()
        warmup = batch if warmup is None else warmup
        stats = []
        for _ in range(n_ticks):
            act = self.model_act(obs)
            out = self.do_actions(act, reset_obs=True)
            d = out["done"].float().repeat(2)
            self.replay.add(obs.reshape(-1, STATE_DIM), act.reshape(-1, ACTION_DIM), out["reward"].reshape(-1),
                            out["obs"].reshape(-1, STATE_DIM), d)
            obs = out["obs_reset"]
            if self.replay.size >= warmup:
                for _ in range(updates_per_tick):
                    # the fused path returns slots of a loss ring: keep copies
                    stats.append(tuple(x.detach().clone() for x in self.replay_update(batch)))
            self._refresh_actor_pack()
        return stats

    def tick_graph(self, batch=256, updates_per_tick=1, ticks_per_graph=2, warmup=3, overlap=None):
        """The replay-rule tick of `train_ticks` captured as ONE hipGraph.

        One replay runs `ticks_per_graph` ticks: per tick the fused actor
        kernel (noise call number on device), the fused env step with
        obs/reward/auto-reset into static buffers, a device-side-head insert of
        the 2N transitions, `updates_per_tick` critic + actor updates on
        device-side samples (capturable fused Adam), the soft target update and
        the actor repack.  Every per-tick quantity (ring head and size, step
        and noise counters, RNG offsets) lives on device, so replays continue
        the eager trajectory's semantics.  Returns a TickGraph; `.run(n)`
        replays n times.

        Several ranks (multi_rank "grad" / "shared"): mode "full" captures the
        RCCL collectives (gradient all-reduce, shared-sample all-gather) inside
        the graph (backend nccl); mode "segmented" cuts the capture at every
        collective and replays graph segments with the collectives issued
        between them (any backend, e.g. gloo).  Default: "full" for nccl,
        "segmented" otherwise; SK_TICKGRAPH_MODE overrides.

        The tick form (tick_form; overlap= or SK_TICK_OVERLAP): by default the
        sequential tick in the reference's order (the update draws after the
        tick's insert).  overlap="auto" opts into the overlapped ticks: from
        TICK_OVERLAP_MIN_ENVS games on one rank the acting launches run beside
        the update on a second stream; below that (and with multi_rank "grad")
        with the fp32 kernels, inside the critic's backward launch.  Either way
        the overlapped update draws from the rows inserted before the tick
        (TickGraph.overlap), one tick later than the reference.

        Any ticks_per_graph >= 1: the engine's step counter, the acting
        observation and the overlapped tick's horizon each alternate between
        two slots per tick, so an odd count is captured as two graphs, one
        per starting slot, which run() replays alternately.
        """
        if self.device.type != "cuda":
            raise RuntimeError("tick_graph needs the GPU engine")
        if int(ticks_per_graph) < 1:
            raise ValueError("ticks_per_graph must be >= 1")
        return TickGraph(self, batch, updates_per_tick, int(ticks_per_graph), warmup, overlap)

    # ------------------------------------------------------------ persistence
    def state_dict(self):
        d = dict(actor=self.model_actor.state_dict(), critic=self.model_critic.state_dict(),
                 actor_opt=self.ddpg.optimiser.state_dict(), critic_opt=self.ddpg.critic_optimiser.state_dict(),
                 env=self.game_environment.state_dict())
        if self.ddpg.tau is not None:
            d["target_actor"] = self.ddpg.target_actor.state_dict()
            d["target_critic"] = self.ddpg.target_critic.state_dict()
        return d

    def load_state_dict(self, d):
        self.model_actor.load_state_dict(d["actor"])
        self.model_critic.load_state_dict(d["critic"])
        self.ddpg.optimiser.load_state_dict(d["actor_opt"])
        self.ddpg.critic_optimiser.load_state_dict(d["critic_opt"])
        self.ddpg.optimisers_loaded()
        self.game_environment.load_state_dict(d["env"])
        if self.ddpg.tau is not None and "target_actor" in d:
            self.ddpg.target_actor.load_state_dict(d["target_actor"])
            self.ddpg.target_critic.load_state_dict(d["target_critic"])
        self._params_changed()

    def _params_changed(self):
        """repack every kernel copy of the nets after their parameters were
        replaced outside the update launches"""
        if self.actor_kernel is not None:
            self.actor_kernel.refresh()
        if self.ddpg._fused is not None:
            self.ddpg._fused.pack()
        if self.ddpg._tq is not None:
            self.ddpg._tq.refresh()


TICK_OVERLAP_MIN_ENVS = 16384  # TickGraph's auto overlap threshold (games per rank)


def tick_form(n, batch, capacity, updates_per_tick, multi, fused, f32, fused_act, sliced, env=None):
    """TickGraph's tick form: "sequential" (the reference's order), "streams"
    (the acting launches on a second stream beside the update), "fused" (the
    acting launch inside the critic gradient's backward launch) or "serial"
    (the streams form on one stream, a test reference); see TickGraph.
    SK_TICK_OVERLAP (or tick_graph's overlap=) = 0 (default: the reference's
    draw order, the update sampling the ring after the tick's insert,
    SkillshotLearner.py:316-324) / auto (the overlapped form this function
    picks: streams from TICK_OVERLAP_MIN_ENVS games, else fused where it can)
    / 1 / fused / serial.  The overlapped forms draw the minibatch from the
    ring as it stood before the tick's insert (one tick later than the
    reference; ADVICE r03: opt-in only).  They need the fused update path, one update per tick, the default
    replay mode (SK_FUSED_REPLAY=2) and a ring holding a batch beside the rows
    one insert writes; "fused" the fp32 kernels with the fused act + step
    launch (SK_FUSED_ACT), N % 4 == 0 and the sliced update schedule; several
    ranks run "fused" or "sequential"."""
    env = os.environ if env is None else env
    ov = str(env.get("SK_TICK_OVERLAP", "0"))
    can = (fused and updates_per_tick == 1 and capacity >= batch + 4 * n
           and env.get("SK_FUSED_REPLAY", "2") == "2")
    can_fuse = can and f32 and fused_act and n % 4 == 0 and env.get("SK_FUSED_ACT", "1") != "0" and sliced
    if ov == "auto":
        ov = "1" if n >= TICK_OVERLAP_MIN_ENVS and not multi else ("fused" if can_fuse else "0")
    if multi and ov != "fused":
        ov = "0"
    if not can or ov == "0" or (ov == "fused" and not can_fuse):
        return "sequential"
    return {"fused": "fused", "serial": "serial"}.get(ov, "streams")


class TickGraph:
    """Captured replay-rule ticks (see SkillshotLearner.tick_graph)."""

    def __init__(self, L, batch, updates_per_tick, ticks_per_graph, warmup, overlap=None):
        self.L, self.batch, self.updates, self.ticks = L, batch, updates_per_tick, ticks_per_graph
        self.multi_rank_mode = None
        if L.ddpg.multi():
            mode = os.environ.get("SK_TICKGRAPH_MODE") or (
                "full" if dist.get_backend(L.ddpg.group) == "nccl" else "segmented")
            if mode not in ("full", "segmented"):
                raise ValueError("SK_TICKGRAPH_MODE must be 'full' or 'segmented'")
            self.multi_rank_mode = f"{L.ddpg.multi_rank}/{mode}"
        self._segments = None
        g = L.game_environment
        n = L.n_envs
        dev = L.device
        # the acting observation alternates between two buffers: tick t reads
        # one and the step writes its reset observations into the other (no
        # copy); a replay has an even number of ticks, so it ends where it began
        self._obs = [L.prepare_states().clone(), g.new_obs()]
        self._cur = 0
        self.act = torch.empty((2, n, ACTION_DIM), dtype=torch.float32, device=dev)
        self.out = dict(obs=g.new_obs(), reward=torch.empty((2, n), dtype=torch.float32, device=dev),
                        done=torch.empty(n, dtype=torch.uint8, device=dev),
                        winner=torch.empty(n, dtype=torch.uint8, device=dev), obs_reset=self._obs[1])
        self.stream = torch.cuda.Stream(device=dev)
        self.stream.wait_stream(torch.cuda.current_stream(dev))
        # The overlapped tick (one rank): the acting launches (act + step +
        # ring insert) run on a second stream beside the update, whose
        # minibatch comes from the rows inserted before this tick
        # (ReplayRing.horizon, the insert's rows excluded: the reference's
        # replay draws after the tick's remember, SkillshotLearner.py:316-324,
        # so this sees the ring one tick late); the two streams join before
        # the actor's Adam launch, which rewrites the weights the acting
        # launch reads (_tick_overlap).  SK_TICK_OVERLAP: auto (default) from
        # TICK_OVERLAP_MIN_ENVS games, where the acting launches are long
        # enough to hide the update (config 5 on one GPU: fp32 280 -> 259 us,
        # bf16 130.6 -> 118 us; config 3 neutral, the graph's cross-queue
        # edges cost what the overlap saves: profiles/r03ov_*); 1 / 0 force.
        # (the ring must hold a batch beside the rows one insert overwrites)
        # Below that, with the fp32 kernels (SK_TICK_OVERLAP=fused, auto): the
        # same tick on one stream, the acting launch run by the actor
        # gradient's backward launch in its spare workgroups
        # (sk_actor_grad_f32_step; _tick_fused); SK_TICK_OVERLAP=serial: the
        # same tick with plain launches on one stream (the check that neither
        # form races).
        # Several ranks: the fused form (config 4, multi_rank "grad": each
        # rank draws from its own ring; config 5, "shared": the drawn rows are
        # all-gathered first; the acting tick rides the critic's backward
        # launch, before the gradient all-reduce); else sequential.
        fu = L.ddpg._fused
        self.mode = tick_form(n, batch, L.replay.cap, updates_per_tick, L.ddpg.multi(), fu is not None,
                              fu is not None and fu.f32, getattr(L.actor_kernel, "fused_act_step", False),
                              fu is not None and fu.sliced(batch),
                              env=dict(os.environ, **({} if overlap is None else {"SK_TICK_OVERLAP": str(overlap)})))
        self.overlap = self.mode != "sequential"
        self.fuse_act = self.mode == "fused"
        self.side = torch.cuda.Stream(device=dev) if self.mode == "streams" else None
        # which backward launch carries the acting tick (SK_FUSE_ACT_IN): the
        # critic's (default, the longer of the two) or the actor's
        self.job_in = os.environ.get("SK_FUSE_ACT_IN", "critic")
        if self.fuse_act:
            from . import _capi
            self._job = _capi.SkStepJob()
        else:
            self._job = None
        self._hp = 0  # host parity of the horizon slots
        self._capturing = False
        with torch.cuda.stream(self.stream):
            # fill the ring past one batch plus one tick without updates (the
            # overlapped update samples the rows before the tick's insert),
            # then warm the update path eagerly (allocator pools, Adam state)
            while L.replay.size < batch + (2 * n if self.overlap else 0):
                self._tick(update=False)
            for _ in range(max(warmup, 1)):
                self._tick(update=True)
            if self._cur:  # start the captured ticks from buffer 0
                self._obs[0].copy_(self._obs[1])
                self._cur = 0
            self._hp = 0
        self.stream.synchronize()
        # capture at a synced step counter (both device slots current, host
        # parity 0): run() syncs before replaying, so eager steps between
        # replays cannot leave the captured slot stale
        g.sync_step_counter(ctypes.c_void_p(self.stream.cuda_stream))
        mirror = L.replay.total  # capture records the inserts without running them
        # Every captured tick samples with the same draw numbers (draw0 + u for
        # its u-th update): the ring count in the sample's key already differs
        # per tick, and a host counter advanced during capture would bake
        # numbers that depend on where the ticks are cut into graphs
        self._draw0 = L.replay._draws
        # Every tick flips three two-slot alternations (the engine's step
        # counter slot, the acting observation buffer, the overlapped tick's
        # horizon), so a graph of an odd number of ticks ends in the other
        # slot than it starts in: then a second graph is captured right after
        # the first, starting where the first ends, and run() alternates the
        # two (phase 0 / 1).  An even count needs one graph.
        self._phases = []
        for _ in range(1 if self.ticks % 2 == 0 else 2):
            if self.multi_rank_mode and self.multi_rank_mode.endswith("segmented"):
                self._phases.append(("segments", self._capture_segments()))
                continue
            graph = torch.cuda.CUDAGraph()
            graph.register_generator_state(L.gen)
            # thread-local capture: only this thread's HIP calls are checked
            # against the capture, so RCCL's watchdog thread may keep
            # querying the events of eager collectives from the warm-up
            # (global mode aborted the process when it did, intermittently)
            self._capturing = True
            try:
                with torch.cuda.graph(graph, stream=self.stream, capture_error_mode="thread_local"):
                    for _ in range(self.ticks):
                        self._tick(update=True)
            finally:
                self._capturing = False
            self._phases.append(("graph", graph))
        self.graph = self._phases[0][1] if self._phases[0][0] == "graph" else None
        self._segments = self._phases[0][1] if self._phases[0][0] == "segments" else None
        self._phase = 0  # which graph the next replay runs (the slot the current tick starts in)
        self.stream.synchronize()
        L.replay.total = mirror
        L.replay._draws = (self._draw0 + self.updates) & 0x7FFFFFFF
        self.replays = 0

    def _capture_segments(self):
        """capture the ticks as graph segments cut at every collective:
        returns [graph, fn, graph, fn, ..., graph] (fn = the collective,
        issued eagerly on replay between the segments it separates)"""
        L = self.L
        pool = torch.cuda.graph_pool_handle()
        items = []
        cur = []

        def begin():
            g = torch.cuda.CUDAGraph()
            g.register_generator_state(L.gen)
            g.capture_begin(pool=pool, capture_error_mode="thread_local")
            cur[:] = [g]

        def cut(fn):
            cur[0].capture_end()
            items.append(cur[0])
            items.append(fn)
            begin()

        with torch.cuda.stream(self.stream):
            L.ddpg.collective_hook = cut
            try:
                begin()
                for _ in range(self.ticks):
                    self._tick(update=True)
                cur[0].capture_end()
                items.append(cur[0])
            finally:
                L.ddpg.collective_hook = None
        return items

    @property
    def obs(self):
        """the observation the next replayed tick acts on"""
        return self._obs[getattr(self, "_phase", self._cur)]

    def _act_insert(self, obs, total_copy=None):
        """act -> do_actions -> game_tick -> get_state (SkillshotLearner.py
        :304-314) and the ring insert: the fp32 actor inside the step launch
        (sk_env_act_step: the observations stay on the CU), else the actor
        launch then sk_env_step_insert"""
        L = self.L
        mode = L.exploration
        if getattr(L.actor_kernel, "fused_act_step", False) and os.environ.get("SK_FUSED_ACT", "1") != "0":
            L.game_environment.act_step(L.actor_kernel, obs,
                                        noise_sd=L.param_noise_sd if mode == "param_noise" else 0.0,
                                        action_sd=L.action_noise_sd if mode == "action_noise" else 0.0,
                                        ring=L.replay, out=self.out, actions=self.act, total_copy=total_copy)
            return
        x, a = obs.view(-1, STATE_DIM), self.act.view(-1, ACTION_DIM)
        if L.actor_kernel is not None and mode == "action_noise" and getattr(L.actor_kernel, "fused_action_noise",
                                                                               False):
            L.actor_kernel(x, out=a, action_sd=L.action_noise_sd)
        elif L.actor_kernel is not None:
            L.actor_kernel(x, noise_sd=L.param_noise_sd if mode == "param_noise" else 0.0, out=a)
            if mode == "action_noise":
                a.add_(L.action_noise_sd * torch.randn(a.shape, device=a.device, generator=L.gen))
        else:
            a.copy_(L.model_act(obs).view(-1, ACTION_DIM))
        L.game_environment.step_insert(self.act, obs, L.replay, reward="looking", auto_reset=True, reset_obs=True,
                                       out=self.out, total_copy=total_copy)

    def _tick_overlap(self):
        """one overlapped tick: the acting launches on the side stream, the
        update on this one (see __init__).  The update of a tick of parity p
        keys its minibatch on horizon[p], the row count before the tick's
        insert; the insert's launch writes horizon[1 - p] (its total_copy).  Eager ticks
        set horizon[p] first; a captured replay starts at parity 0 with
        horizon[0] set by run().  Deterministic: the update reads no row and
        no count that the acting launches write."""
        L = self.L
        ring = L.replay
        main = torch.cuda.current_stream(L.device)
        p = self._hp
        if not self._capturing:
            ring.horizon[p].copy_(ring.total_t)
        obs = self._obs[self._cur]
        self.out["obs_reset"] = self._obs[1 - self._cur]
        side = self.side if self.side is not None else main
        side.wait_stream(main)
        with torch.cuda.stream(side):
            self._act_insert(obs, total_copy=ring.horizon[1 - p])
        self._cur ^= 1
        self._hp ^= 1
        L.ddpg.update_overlapped(self.batch, ring.horizon[p], 2 * L.n_envs,
                                 before_actor_adam=lambda: main.wait_stream(side))
        L._refresh_actor_pack()

    def _tick_fused(self):
        """one fused overlapped tick: the acting launch is prepared (not
        issued), the update draws its minibatch from the count before the
        tick's insert (the insert's rows excluded, as _tick_overlap's), and
        the actor gradient's backward launch runs the acting tick beside it,
        before the actor's Adam launch.  Equal, bit for bit, to
        _tick_overlap's tick (tests/test_replay_gpu.py)."""
        L = self.L
        ring = L.replay
        obs = self._obs[self._cur]
        self.out["obs_reset"] = self._obs[1 - self._cur]
        mode = L.exploration
        L.game_environment.act_step(L.actor_kernel, obs, noise_sd=L.param_noise_sd if mode == "param_noise" else 0.0,
                                    action_sd=L.action_noise_sd if mode == "action_noise" else 0.0, ring=ring,
                                    out=self.out, actions=self.act, job=self._job)
        self._cur ^= 1
        L.ddpg.update_overlapped(self.batch, ring.total_t, 2 * L.n_envs, step_job=self._job, job_in=self.job_in)
        L._refresh_actor_pack()

    def _tick(self, update):
        L = self.L
        if getattr(self, "_draw0", None) is not None:  # a captured tick (see __init__)
            L.replay._draws = self._draw0
        if update and self.fuse_act:
            return self._tick_fused()
        if update and self.overlap:
            return self._tick_overlap()
        obs = self._obs[self._cur]
        self.out["obs_reset"] = self._obs[1 - self._cur]
        x = obs.view(-1, STATE_DIM)
        a = self.act.view(-1, ACTION_DIM)
        mode = L.exploration
        fused = os.environ.get("SK_FUSED_REPLAY", "2")
        if (fused == "2" and getattr(L.actor_kernel, "fused_act_step", False)
                and os.environ.get("SK_FUSED_ACT", "1") != "0"):
            self._act_insert(obs)
            self._cur ^= 1
            if update:
                for _ in range(self.updates):
                    L.ddpg.update_sampled(self.batch)
                L._refresh_actor_pack()
            return
        if L.actor_kernel is not None and mode == "action_noise" and getattr(L.actor_kernel, "fused_action_noise",
                                                                               False):
            L.actor_kernel(x, out=a, action_sd=L.action_noise_sd)
        elif L.actor_kernel is not None:
            L.actor_kernel(x, noise_sd=L.param_noise_sd if mode == "param_noise" else 0.0, out=a)
            if mode == "action_noise":
                a.add_(L.action_noise_sd * torch.randn(a.shape, device=a.device, generator=L.gen))
        else:
            a.copy_(L.model_act(obs).view(-1, ACTION_DIM))
        # SK_FUSED_REPLAY (A/B): 2 (default) the ring insert inside the step
        # launch and the minibatch drawn inside the critic step's; 1 the
        # insert and the first minibatch in one launch after the step; 0 the
        # insert and the sample as their own launches.  SK_FUSED_ACT=0 keeps
        # the actor forward as its own launch (fp32 actor, mode 2)
        if fused == "2":
            L.game_environment.step_insert(self.act, obs, L.replay, reward="looking", auto_reset=True,
                                           reset_obs=True, out=self.out)
            self._cur ^= 1
            if update:
                for _ in range(self.updates):
                    L.ddpg.update_sampled(self.batch)
                L._refresh_actor_pack()
            return
        o = L.game_environment.step(self.act, obs=True, reward="looking", auto_reset=True, reset_obs=True,
                                    out=self.out)
        # per game: row r of the [2N] rows takes game r % N
        rows = (x, a, o["reward"].view(-1), o["obs"].view(-1, STATE_DIM), o["done"])
        self._cur ^= 1
        if update and self.updates > 0 and fused != "0":
            # the insert and the first update's minibatch in one launch
            # (SK_FUSED_REPLAY=0: the two launches, for A/B)
            L.ddpg.update_batch(*L.replay.add_sample_dev(*rows, self.batch))
            for _ in range(self.updates - 1):
                L.ddpg.replay_update(self.batch, device_sampling=True)
            L._refresh_actor_pack()
        else:
            L.replay.add_dev(*rows)
            if update:
                for _ in range(self.updates):
                    L.ddpg.replay_update(self.batch, device_sampling=True)
                L._refresh_actor_pack()

    def run(self, n=1):
        """n graph replays (n * ticks_per_graph ticks) on the caller's current
        stream.  Work queued on `self.stream` (the capture stream) before the
        call is waited for first.  The replays are not put on the capture
        stream: the form that did so ended with the caller's stream waiting
        on it, and that wait, pending in another hardware queue while the
        replays ran, slowed every replayed tick by ~5 us (config 3 52.0 ->
        57.4 us per tick; tools/graph_host_rate.py, profiles/r06at_tickgraph_stream/)."""
        cur = torch.cuda.current_stream(self.L.device)
        cur.wait_stream(self.stream)
        # both step slots current: the graph of either phase reads its own
        self.L.game_environment.sync_step_counter(ctypes.c_void_p(cur.cuda_stream))
        if self.overlap:  # the first replayed update samples the current count
            self.L.replay.horizon[self._phase].copy_(self.L.replay.total_t)
        for _ in range(n):
            kind, g = self._phases[self._phase]
            if kind == "graph":
                g.replay()  # on the current stream
            else:
                for it in g:
                    if callable(it) and not isinstance(it, torch.cuda.CUDAGraph):
                        it()
                    else:
                        it.replay()
            self._phase = (self._phase + self.ticks) % 2
        self.replays += n
        # host mirrors of the ring (2N rows per tick)
        r, rows = self.L.replay, n * self.ticks * 2 * self.obs.shape[1]
        r.total += rows
