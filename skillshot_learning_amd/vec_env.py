"""VecSkillshotGame — N Skillshot games stepped on one MI355X by libskillshot.

State lives in HBM as torch tensors (the struct-of-arrays layout of
include/skillshot.h) that the C engine is attached to, so observations,
rewards and the state itself are torch tensors with no copies.  Every method
is the batched form of a reference method (cited per method); the fused
`step` is the learner's whole per-tick protocol (SkillshotLearner.py:302-324)
in one kernel launch.
"""
import ctypes

import numpy as np
import torch

from . import _capi
from ._capi import SkillshotError, check

PLANES = (("pos", torch.int32, 4), ("rot", torch.float64, 2), ("qpos", torch.int32, 4),
          ("qrot", torch.float64, 2), ("qcdage", torch.int32, 4), ("misc", torch.int32, 2))

REWARD_KINDS = {"looking": _capi.SK_REWARD_LOOKING, "simple": _capi.SK_REWARD_SIMPLE}

# get_state per-player key order (SkillshotGame.py:145-163); sk_env_features columns
FEATURE_KEYS = ("player_grad", "player_x_dir", "player_path_dist_opponent", "player_dist_opponent",
                "player_pos_x", "player_pos_y", "player_rotation", "projectile_cooldown",
                "projectile_grad", "projectile_x_dir", "projectile_path_dist_opponent",
                "projectile_pos_x", "projectile_pos_y", "projectile_rotation", "projectile_age",
                "projectile_valid", "projectile_dist_opponent", "projectile_future_collision_opponent")


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _resolve_device(device):
    """cuda[:i] -> the gfx950 engine on that device; cpu -> libskillshot's CPU
    backend (device = -1, csrc/sk_host.cpp), chosen explicitly, never as a
    fallback: a cuda request without a GPU raises."""
    dev = torch.device(device)
    if dev.type == "cpu":
        return dev
    if dev.type != "cuda":
        raise SkillshotError(f"VecSkillshotGame runs on a gfx950 GPU or the CPU backend, not {dev}")
    if not torch.cuda.is_available():
        raise SkillshotError("no GPU visible (use device='cpu' for libskillshot's CPU backend)")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    return torch.device("cuda", idx)


class VecSkillshotGame:
    """N independent games (the reference SkillshotGame, batched).

    n_envs      games on this device
    env_offset  global id of game 0 (multi-GPU sharding; RNG is keyed by global id)
    seed        Philox key for random starts / random-policy actions
    tick_limit  episode length cap (SkillshotLearner.model_param_game_tick_limit, :62)
    random_positions  use random starts on reset (SkillshotLearner.use_random_start, :44)
    """

    def __init__(self, n_envs, device="cuda", seed=0, env_offset=0, tick_limit=2000,
                 random_positions=True, config=None):
        self.device = _resolve_device(device)
        self.is_cpu = self.device.type == "cpu"
        self.n = int(n_envs)
        if self.n <= 0:
            raise ValueError("n_envs must be > 0")
        self.seed = int(seed)
        self.env_offset = int(env_offset)
        self.tick_limit = int(tick_limit)
        self.random_positions = bool(random_positions)
        self._L = _capi.load()
        # one allocation, the planes back to back (88 B per game, every plane
        # 16-byte aligned): the multi-tick kernels address all six through
        # one buffer resource with 32-bit offsets (sk_env_step_multi)
        self._state_buf = torch.zeros(88 * self.n, dtype=torch.uint8, device=self.device)
        off = 0
        for name, dt, w in PLANES:
            nbytes = self.n * w * torch.empty((), dtype=dt).element_size()
            setattr(self, name, self._state_buf[off:off + nbytes].view(dt).view(self.n, w))
            off += nbytes
        view = _capi.SkStateView(self.n, *[getattr(self, name).data_ptr() for name, _, _ in PLANES])
        cfg = config if config is not None else _capi.default_config()
        self.config = cfg
        h = ctypes.c_void_p()
        self._sync()
        check(self._L.sk_env_attach(ctypes.byref(h), ctypes.byref(view), self.env_offset, self.seed,
                                    -1 if self.is_cpu else self.device.index, ctypes.byref(cfg)))
        self._h = h
        cp = ctypes.c_void_p()
        check(self._L.sk_env_counters_ptr(self._h, ctypes.byref(cp)))
        self._counters_ptr = cp.value
        self.reset(random_positions=False)

    # ------------------------------------------------------------------ utils
    def _stream(self):
        if self.is_cpu:
            return None
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _sync(self):
        if not self.is_cpu:
            torch.cuda.synchronize(self.device)

    def close(self):
        if getattr(self, "_h", None):
            self._sync()
            self._L.sk_env_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def step_counter(self):
        v = ctypes.c_uint64()
        check(self._L.sk_env_get_step_counter(self._h, ctypes.byref(v)))
        return v.value

    @step_counter.setter
    def step_counter(self, value):
        check(self._L.sk_env_set_step_counter(self._h, int(value)))

    def sync_step_counter(self, stream=None):
        """Stream-ordered: both device step slots take the current value, so
        graphs captured after this call replay with correct RNG keys after any
        mix of eager launches (sk_env_sync_step_counter)."""
        check(self._L.sk_env_sync_step_counter(self._h, stream if stream is not None else self._stream()))

    def state_dict(self):
        """Host copy of the state planes (engine layout) + RNG counter."""
        d = {name: getattr(self, name).cpu().numpy().copy() for name, _, _ in PLANES}
        d["step_counter"] = self.step_counter
        return d

    def load_state_dict(self, d):
        self._sync()
        for name, dt, w in PLANES:
            src = torch.as_tensor(np.asarray(d[name]).reshape(self.n, w)).to(dt)
            getattr(self, name).copy_(src)
        if "step_counter" in d:
            self.step_counter = int(d["step_counter"])
        self._sync()

    def get_board(self, index=0):
        """SkillshotGame.get_board (SkillshotGame.py:36-56) of game `index`:
        int64 [250, 250], [x, y] indexing (host rasteriser, visualisation only)."""
        from .game import rasterize_board
        i = int(index)
        pos = self.pos[i].cpu().tolist()
        qpos = self.qpos[i].cpu().tolist()
        rot = self.rot[i].cpu().tolist()
        flags = int(self.misc[i, 1].item()) & 0xFFFFFFFF
        return rasterize_board(np.zeros((250, 250), dtype=np.int64), [pos[0:2], pos[2:4]], rot,
                               [qpos[0:2], qpos[2:4]], [flags & 0xFF, (flags >> 8) & 0xFF])

    # convenience decoded views -------------------------------------------
    @property
    def ticks(self):
        return self.misc[:, 0]

    @property
    def flags(self):
        return self.misc[:, 1]

    @property
    def game_live(self):
        return ((self.misc[:, 1] >> 16) & 0xFF).to(torch.bool)

    @property
    def winner_id(self):
        return ((self.misc[:, 1] >> 24) & 0xFF).to(torch.uint8)

    @property
    def projectile_valid(self):
        f = self.misc[:, 1]
        return torch.stack([(f & 0xFF), (f >> 8) & 0xFF], -1).to(torch.bool)

    def counters(self, stream=None):
        """Episode counters (dones, hits by id, tick sum) accumulated on device
        by the step kernels' wavefront ballots (read on `stream`, default
        torch's current one: pass the stream the steps ran on)."""
        c = _capi.SkCounters()
        check(self._L.sk_env_read_counters(self._h, ctypes.byref(c), stream if stream is not None else self._stream()))
        return dict(dones=c.dones, hits_p1=c.hits_p1, hits_p2=c.hits_p2, ticks_sum=c.ticks_sum)

    def clear_counters(self, stream=None):
        """Zero the episode counters, ordered on `stream` (default torch's
        current one: pass the stream the steps run on)."""
        check(self._L.sk_env_clear_counters(self._h, stream if stream is not None else self._stream()))

    # ------------------------------------------------------------ reference API
    def reset(self, mask=None, random_positions=None):
        """SkillshotGame.game_reset (SkillshotGame.py:168-169) for masked envs."""
        rp = self.random_positions if random_positions is None else bool(random_positions)
        m = None if mask is None else self._u8(mask)
        check(self._L.sk_env_reset(self._h, _ptr(m), int(rp), self._stream()))

    def move_direction(self, player_id, speeds):
        """Player.move_direction_float (Player.py:57-68) for one player of every env."""
        v, s = self._f64_or_scalar(speeds)
        check(self._L.sk_player_move_direction(self._h, int(player_id), _ptr(v), s, self._stream()))

    def move_look(self, player_id, angles):
        """Player.move_look_float (Player.py:33-39)."""
        v, s = self._f64_or_scalar(angles)
        check(self._L.sk_player_move_look(self._h, int(player_id), _ptr(v), s, self._stream()))

    def move_discrete(self, player_id, kind, mask=None):
        """Keyboard moves (Player.py:27-55): kind 0 forwards, 1 backwards, 2 look left, 3 look right."""
        m = None if mask is None else self._u8(mask)
        check(self._L.sk_player_move_discrete(self._h, int(player_id), int(kind), _ptr(m), self._stream()))

    def shoot(self, player_id, mask=None):
        """Player.move_shoot_projectile (Player.py:78-89) for masked envs."""
        m = None if mask is None else self._u8(mask)
        check(self._L.sk_player_shoot(self._h, int(player_id), _ptr(m), self._stream()))

    def projectile_move(self, player_id, tick=True, mask=None):
        """Projectile.tick (Projectile.py:49-53) or, with tick=False, move_forwards (:38-47)."""
        m = None if mask is None else self._u8(mask)
        check(self._L.sk_projectile_move(self._h, int(player_id), int(bool(tick)), _ptr(m), self._stream()))

    def check_collision(self, hit_out=None):
        """SkillshotGame.check_collision (SkillshotGame.py:58-94); returns u8[N] id of the player hit (0 = none)."""
        h = hit_out if hit_out is not None else torch.empty(self.n, dtype=torch.uint8, device=self.device)
        check(self._L.sk_game_check_collision(self._h, _ptr(h), self._stream()))
        return h

    def game_tick(self):
        """SkillshotGame.game_tick (SkillshotGame.py:115-122)."""
        check(self._L.sk_game_tick(self._h, self._stream()))

    def features(self, out=None):
        """get_state() numerics (SkillshotGame.py:136-166): float64 [N, 2, 18] in FEATURE_KEYS order."""
        f = out if out is not None else torch.empty((self.n, 2, 18), dtype=torch.float64, device=self.device)
        check(self._L.sk_env_features(self._h, _ptr(f), self._stream()))
        return f

    def observe(self, reward="looking", obs_out=None, reward_out=None):
        """prepare_states (SkillshotLearner.py:512-543) -> obs [2,N,12] f32 and
        calculate_rewards_<reward> (:575-603) -> reward [2,N] f32 of the current state."""
        obs = obs_out if obs_out is not None else self.new_obs()
        rew = reward_out if reward_out is not None else torch.empty((2, self.n), dtype=torch.float32,
                                                                      device=self.device)
        check(self._L.sk_env_observe(self._h, _ptr(obs), _ptr(rew), REWARD_KINDS[reward], self._stream()))
        return obs, rew

    # ---------------------------------------------------------------- hot path
    def new_obs(self):
        return torch.empty((2, self.n, 12), dtype=torch.float32, device=self.device)

    def step(self, actions, obs=True, reward="looking", auto_reset=True, reset_obs=False, out=None):
        """One learner tick for every env (SkillshotLearner.py:302-324), one launch.

        actions: float32 [2, N, 2] (player, env, {speed, look}).
        Returns dict(obs [2,N,12] | None, reward [2,N] | None, done u8[N], winner u8[N],
        obs_reset [2,N,12] | None): obs/reward/done/winner describe the post-tick
        (terminal) state; with auto_reset the done envs are then reset and
        obs_reset holds the obs the next tick acts on.
        """
        a = self._actions(actions)
        o = out or {}
        obs_t = (o.get("obs") if o.get("obs") is not None else self.new_obs()) if obs else None
        rew_t = (o.get("reward") if o.get("reward") is not None else
                 torch.empty((2, self.n), dtype=torch.float32, device=self.device)) if obs else None
        done = o.get("done") if o.get("done") is not None else torch.empty(self.n, dtype=torch.uint8,
                                                                            device=self.device)
        win = o.get("winner") if o.get("winner") is not None else torch.empty(self.n, dtype=torch.uint8,
                                                                               device=self.device)
        obs_r = (o.get("obs_reset") if o.get("obs_reset") is not None else self.new_obs()) if reset_obs else None
        check(self._L.sk_env_step(self._h, _ptr(a), _ptr(obs_t), _ptr(rew_t), REWARD_KINDS[reward], _ptr(done),
                                  _ptr(win), self.tick_limit, int(bool(auto_reset)), int(self.random_positions),
                                  _ptr(obs_r), self._stream()))
        return dict(obs=obs_t, reward=rew_t, done=done, winner=win, obs_reset=obs_r)

    def step_insert(self, actions, acting_obs, ring, reward="looking", auto_reset=True, reset_obs=True, out=None,
                    total_copy=None):
        """`step` (obs and reward on) and the replay ring's insert of the tick's
        2N transitions (acting_obs[r], actions[r], reward[r], obs[r],
        done[r % N]) in ONE launch (sk_env_step_insert): equal, bit for bit,
        to step(...) followed by ring.add_dev(acting_obs, actions, reward,
        obs, done).  ring: learner.ReplayRing on this env's device;
        total_copy: an int64 element that receives the new row count too."""
        a = self._actions(actions)
        o = out or {}
        obs_t = o.get("obs") if o.get("obs") is not None else self.new_obs()
        rew_t = o.get("reward") if o.get("reward") is not None else torch.empty((2, self.n), dtype=torch.float32,
                                                                                device=self.device)
        done = o.get("done") if o.get("done") is not None else torch.empty(self.n, dtype=torch.uint8,
                                                                            device=self.device)
        win = o.get("winner") if o.get("winner") is not None else torch.empty(self.n, dtype=torch.uint8,
                                                                               device=self.device)
        obs_r = (o.get("obs_reset") if o.get("obs_reset") is not None else self.new_obs()) if reset_obs else None
        s = acting_obs.float().contiguous()
        if s.numel() != 2 * self.n * 12:
            raise ValueError("acting_obs must hold [2, N, 12] floats")
        check(self._L.sk_env_step_insert(self._h, _ptr(a), _ptr(obs_t), _ptr(rew_t), REWARD_KINDS[reward],
                                         _ptr(done), _ptr(win), self.tick_limit, int(bool(auto_reset)),
                                         int(self.random_positions), _ptr(obs_r), _ptr(s), _ptr(ring.buf), ring.cap,
                                         _ptr(ring.total_t), _ptr(ring.arrivals()), _ptr(total_copy),
                                         self._stream()))
        ring.total += 2 * self.n  # host mirror (exact while the row count is fixed)
        return dict(obs=obs_t, reward=rew_t, done=done, winner=win, obs_reset=obs_r)

    def act_step(self, actor, acting_obs, noise_sd=0.0, action_sd=0.0, ring=None, reward="looking", auto_reset=True,
                 reset_obs=True, out=None, actions=None, total_copy=None, job=None):
        """The self-play tick's act + step (+ ring insert) in ONE launch
        (sk_env_act_step): `actor` (actor_kernel.ActorKernel32, the fp32
        actor) acts on acting_obs [2, N, 12] for both players of every game
        with parameter noise noise_sd and/or action noise action_sd, and the
        step runs on those actions; equal, bit for bit, to actor(...) with
        32-row tiles followed by step_insert (ring given; total_copy as
        step_insert's) or step.  job (_capi.SkStepJob): prepare the launch
        into it instead (sk_env_act_step_job; run by the actor step's
        backward launch, update_kernel.actor_step(step_job=job)).  Returns
        step's dict plus `actions` [2, N, 2]."""
        o = out or {}
        obs_t = o.get("obs") if o.get("obs") is not None else self.new_obs()
        rew_t = o.get("reward") if o.get("reward") is not None else torch.empty((2, self.n), dtype=torch.float32,
                                                                                device=self.device)
        done = o.get("done") if o.get("done") is not None else torch.empty(self.n, dtype=torch.uint8,
                                                                            device=self.device)
        win = o.get("winner") if o.get("winner") is not None else torch.empty(self.n, dtype=torch.uint8,
                                                                               device=self.device)
        obs_r = (o.get("obs_reset") if o.get("obs_reset") is not None else self.new_obs()) if reset_obs else None
        act = actions if actions is not None else torch.empty((2, self.n, 2), dtype=torch.float32, device=self.device)
        s = acting_obs.float().contiguous()
        if s.numel() != 2 * self.n * 12 or act.numel() != 4 * self.n or not act.is_contiguous():
            raise ValueError("acting_obs must hold [2, N, 12] floats, actions [2, N, 2] (contiguous)")
        ring_args = ((_ptr(ring.buf), ring.cap, _ptr(ring.total_t), _ptr(ring.arrivals()), _ptr(total_copy))
                     if ring is not None else (None, 0, None, None, None))
        pack = actor.ensure_pack()
        args = (self._h, _ptr(actor.flat), _ptr(pack), _ptr(s), _ptr(act), float(noise_sd), float(action_sd), actor.seed,
                _ptr(actor._ctr), _ptr(obs_t), _ptr(rew_t), REWARD_KINDS[reward], _ptr(done), _ptr(win),
                self.tick_limit, int(bool(auto_reset)), int(self.random_positions), _ptr(obs_r), *ring_args)
        if job is not None:
            check(self._L.sk_env_act_step_job(*args, ctypes.byref(job)))
        else:
            check(self._L.sk_env_act_step(*args, self._stream()))
        if ring is not None:
            ring.total += 2 * self.n  # host mirror
        return dict(obs=obs_t, reward=rew_t, done=done, winner=win, obs_reset=obs_r, actions=act)

    def act_episode(self, actor, start_obs, n_ticks=None, noise_sd=0.0, action_sd=0.0, reward="looking",
                    out=None):
        """The reference rule's episode collection in ONE launch
        (sk_env_act_episode; SkillshotLearner.model_train :289-318 for every
        game): from the current state every game plays until it ends (hit or
        tick limit), acting with `actor` (ActorKernel32) with fresh noise per
        tick.  start_obs [2, N, 12]: the observation of the current state.
        Returns dict(states [T+1, 2, N, 12], actions [T, 2, N, 2], rewards
        [T, 2, N], lengths int32 [N]); rows t < lengths[i] are game i's
        episode.  T = n_ticks (default: the tick limit); a game still live
        after T ticks continues in the next call (from states[T]).  The
        device step counter and the actor's noise call number (actor.calls)
        advance on device by max(lengths), the ticks the per-tick loop would
        have run."""
        T = int(self.tick_limit if n_ticks is None else n_ticks)
        o = out or {}
        st = o.get("states")
        if st is None or st.shape[0] < T + 1:
            st = torch.empty((T + 1, 2, self.n, 12), dtype=torch.float32, device=self.device)
        ac = o.get("actions")
        if ac is None or ac.shape[0] < T:
            ac = torch.empty((T, 2, self.n, 2), dtype=torch.float32, device=self.device)
        rw = o.get("rewards")
        if rw is None or rw.shape[0] < T:
            rw = torch.empty((T, 2, self.n), dtype=torch.float32, device=self.device)
        ln = o.get("lengths")
        if ln is None:
            ln = torch.empty(self.n, dtype=torch.int32, device=self.device)
        st[0].copy_(start_obs.reshape(2, self.n, 12))
        pack = actor.ensure_pack()
        check(self._L.sk_env_act_episode(self._h, _ptr(actor.flat), _ptr(pack), _ptr(st), _ptr(ac), _ptr(rw),
                                         _ptr(ln), T, float(noise_sd), float(action_sd), actor.seed,
                                         _ptr(actor._ctr), REWARD_KINDS[reward], self.tick_limit, self._stream()))
        return dict(states=st[:T + 1], actions=ac[:T], rewards=rw[:T], lengths=ln)

    def step_raw(self, actions_ptr, done_ptr=None, obs_ptr=None, reward_ptr=None, winner_ptr=None,
                 auto_reset=True, stream=None):
        """Pointer-level fused step (bench / graph capture; no allocation)."""
        check(self._L.sk_env_step(self._h, actions_ptr, obs_ptr, reward_ptr, 0, done_ptr, winner_ptr,
                                  self.tick_limit, int(bool(auto_reset)), int(self.random_positions), None,
                                  stream if stream is not None else self._stream()))

    def step_multi(self, actions, n_ticks=None, slab0=0, done=None, winner=None, record=False, auto_reset=True,
                   stream=None):
        """n_ticks step-only learner ticks (SkillshotLearner.py:302-318: do_actions x2,
        game_tick, done, random restart) in ONE launch (sk_env_step_multi).

        actions: float32 [R, 2, N, 2], a ring of R per-tick slabs; tick t acts on
        slab (slab0 + t) % R.  n_ticks defaults to R.  done / winner: u8 [N]
        (the last tick's) or, with record=True, [n_ticks, N] (every tick's).
        Equal bit for bit to n_ticks `step(actions[s], obs=False)` calls."""
        a = torch.as_tensor(actions, device=self.device)
        if a.dtype != torch.float32 or not a.is_contiguous() or a.dim() != 4 or tuple(a.shape[1:]) != (2, self.n, 2):
            raise ValueError(f"actions must be contiguous float32 [R, 2, {self.n}, 2]")
        R = a.shape[0]
        T = R if n_ticks is None else int(n_ticks)
        rows = T if record else 1
        if done is None:
            done = torch.empty((rows, self.n), dtype=torch.uint8, device=self.device)
        if winner is None:
            winner = torch.empty((rows, self.n), dtype=torch.uint8, device=self.device)
        for t in (done, winner):
            if t.numel() < rows * self.n or t.dtype != torch.uint8 or not t.is_contiguous():
                raise ValueError(f"done / winner must be contiguous uint8 with {rows} x {self.n} elements")
        check(self._L.sk_env_step_multi(self._h, _ptr(a), R, int(slab0) % R, T, _ptr(done), _ptr(winner),
                                        self.n if record else 0, self.tick_limit, int(bool(auto_reset)),
                                        int(self.random_positions), stream if stream is not None else self._stream()))
        return done.view(rows, self.n) if record else done.view(-1)[: self.n], \
            winner.view(rows, self.n) if record else winner.view(-1)[: self.n]

    def step_multi_obs(self, actions, n_ticks=None, slab0=0, out_slabs=None, out0=0, reward="looking",
                       auto_reset=True, out=None, stream=None):
        """n_ticks ticks of the FULL contract (SkillshotLearner.py:302-324 with
        the actions given: do_actions x2, game_tick, prepare_states and the
        reward of the post-tick state, done, random restart) in ONE launch
        (sk_env_step_multi_obs).

        actions: float32 [R, 2, N, 2], tick t acting on slab (slab0 + t) % R;
        tick t writes output slab (out0 + t) % out_slabs (out_slabs defaults to
        n_ticks: one slab per tick) of obs [S, 2, N, 12], reward [S, 2, N],
        done / winner [S, N].  Equal bit for bit to n_ticks
        `step(actions[s], obs=True, reward=reward)` calls."""
        a = torch.as_tensor(actions, device=self.device)
        if a.dtype != torch.float32 or not a.is_contiguous() or a.dim() != 4 or tuple(a.shape[1:]) != (2, self.n, 2):
            raise ValueError(f"actions must be contiguous float32 [R, 2, {self.n}, 2]")
        R = a.shape[0]
        T = R if n_ticks is None else int(n_ticks)
        S = T if out_slabs is None else int(out_slabs)
        if out is None:
            out = dict(obs=torch.empty((S, 2, self.n, 12), dtype=torch.float32, device=self.device),
                       reward=torch.empty((S, 2, self.n), dtype=torch.float32, device=self.device),
                       done=torch.empty((S, self.n), dtype=torch.uint8, device=self.device),
                       winner=torch.empty((S, self.n), dtype=torch.uint8, device=self.device))
        for k, shape in (("obs", (S, 2, self.n, 12)), ("reward", (S, 2, self.n)), ("done", (S, self.n)),
                         ("winner", (S, self.n))):
            t = out.get(k)
            if t is not None and (tuple(t.shape) != shape or not t.is_contiguous()):
                raise ValueError(f"{k} must be contiguous {shape}")
        check(self._L.sk_env_step_multi_obs(self._h, _ptr(a), R, int(slab0) % R, T, _ptr(out.get("obs")),
                                            _ptr(out.get("reward")), REWARD_KINDS[reward], _ptr(out.get("done")),
                                            _ptr(out.get("winner")), S, int(out0) % S, self.tick_limit,
                                            int(bool(auto_reset)), int(self.random_positions),
                                            stream if stream is not None else self._stream()))
        return out

    def step_multi_raw(self, actions_ptr, ring, slab0, n_ticks, done_ptr=None, winner_ptr=None, out_stride=0,
                       auto_reset=True, stream=None):
        """Pointer-level sk_env_step_multi (bench / graph capture; no allocation)."""
        check(self._L.sk_env_step_multi(self._h, actions_ptr, int(ring), int(slab0), int(n_ticks), done_ptr,
                                        winner_ptr, int(out_stride), self.tick_limit, int(bool(auto_reset)),
                                        int(self.random_positions), stream if stream is not None else self._stream()))

    def gen_random_actions(self, n_ticks, out=None):
        """Random-policy actions float32 [n_ticks, 2, N, 2] (config 2 synthetic input)."""
        a = out if out is not None else torch.empty((n_ticks, 2, self.n, 2), dtype=torch.float32,
                                                    device=self.device)
        check(self._L.sk_gen_random_actions(self._h, _ptr(a), int(n_ticks), self._stream()))
        return a

    def rollout_random(self, n_ticks):
        """n_ticks random-policy ticks with auto-reset, one launch, state in registers."""
        check(self._L.sk_env_rollout_random(self._h, int(n_ticks), self.tick_limit, self._stream()))

    # ---------------------------------------------------------------- helpers
    def _u8(self, mask):
        m = torch.as_tensor(mask, device=self.device)
        if m.dtype != torch.uint8:
            m = m.to(torch.uint8)
        m = m.contiguous()
        if m.numel() != self.n:
            raise ValueError("mask must have n_envs elements")
        return m

    def _f64_or_scalar(self, x):
        if isinstance(x, (int, float)):
            return None, float(x)
        t = torch.as_tensor(x, device=self.device).to(torch.float64).contiguous()
        if t.numel() == 1:
            return None, float(t.item())
        if t.numel() != self.n:
            raise ValueError("need one value per env")
        return t, 0.0

    def _actions(self, actions):
        a = torch.as_tensor(actions, device=self.device)
        if a.dtype != torch.float32:
            a = a.to(torch.float32)
        a = a.contiguous()
        if tuple(a.shape) != (2, self.n, 2):
            raise ValueError(f"actions must be float32 [2, {self.n}, 2], got {tuple(a.shape)}")
        return a
