"""ctypes binding of the CPU oracle (oracle/skillshot_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker / the timed CPU baseline,
never as the product path (the product is skillshot_learning_amd/, which has
no CPU fallback).

The oracle is pinned against golden vectors produced by running the reference
game core (tests/golden/make_golden.py -> tests/golden/*.npz, checked in
tests/test_oracle_golden.py).  State arrays use the engine's HBM layout
(include/skillshot.h) as numpy arrays:
    pos int32[N,4], rot f64[N,2], qpos int32[N,4], qrot f64[N,2],
    qcdage int32[N,4], misc int32[N,2]  (ticks, flags)
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SK_ORACLE_LIB: a differently built copy (the sanitizer run, tools/sanitize.sh)
_LIB_PATH = os.environ.get("SK_ORACLE_LIB") or os.path.join(_HERE, "_build", "libskillshot_oracle.so")
_lib = None

FIELDS = (("pos", np.int32, 4), ("rot", np.float64, 2), ("qpos", np.int32, 4),
          ("qrot", np.float64, 2), ("qcdage", np.int32, 4), ("misc", np.int32, 2))


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.environ.get("SK_ORACLE_LIB") and (not os.path.exists(_LIB_PATH) or (
                os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "skillshot_oracle.c")))):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        view = [P] * 6
        i64, i32, u64, f64 = ctypes.c_int64, ctypes.c_int32, ctypes.c_uint64, ctypes.c_double
        L.orc_reset.argtypes = view + [i64, P, i32, u64, i64, u64]
        L.orc_move_direction.argtypes = view + [i64, i32, P, f64]
        L.orc_move_look.argtypes = view + [i64, i32, P, f64]
        L.orc_move_discrete.argtypes = view + [i64, i32, i32, P]
        L.orc_shoot.argtypes = view + [i64, i32, P]
        L.orc_game_tick.argtypes = view + [i64]
        L.orc_projectile_move.argtypes = view + [i64, i32, i32, P]
        L.orc_check_collision.argtypes = view + [i64, P]
        L.orc_features.argtypes = view + [i64, P]
        L.orc_observe.argtypes = view + [i64, P, P, i32]
        L.orc_step.argtypes = view + [i64, P, P, P, i32, P, P, i32, i32, i32, P, u64, i64, u64, P]
        L.orc_gen_random_actions.argtypes = [i64, P, i32, u64, i64, u64]
        L.orc_rollout_random.argtypes = view + [i64, i32, i32, u64, i64, u64, P]
        L.orc_philox4x32_10.argtypes = [P, P, P]
        L.orc_max_dist.restype = f64
        L.orc_u32_to_action.argtypes = [ctypes.c_uint32]
        L.orc_u32_to_action.restype = ctypes.c_float
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def pack_flags(qvalid, live, winner):
    qvalid = np.asarray(qvalid, dtype=np.uint32)
    return ((qvalid[..., 0] & 0xFF) | ((qvalid[..., 1] & 0xFF) << 8) |
            ((np.asarray(live, np.uint32) & 0xFF) << 16) |
            ((np.asarray(winner, np.uint32) & 0xFF) << 24)).astype(np.uint32).view(np.int32)


def unpack_flags(flags):
    f = np.asarray(flags).astype(np.int64) & 0xFFFFFFFF
    return dict(qvalid=np.stack([f & 0xFF, (f >> 8) & 0xFF], -1).astype(np.uint8),
                live=((f >> 16) & 0xFF).astype(np.uint8), winner=((f >> 24) & 0xFF).astype(np.uint8))


class OracleState:
    """A batch of N envs in the engine layout, stepped by the C oracle."""

    def __init__(self, n, seed=0, env_offset=0):
        self.n = int(n)
        self.seed = int(seed)
        self.env_offset = int(env_offset)
        self.step_counter = 0
        for name, dt, w in FIELDS:
            setattr(self, name, np.zeros((self.n, w), dtype=dt))
        self.counters = np.zeros(4, dtype=np.uint64)
        self.reset(random_positions=False)

    # -- helpers
    def _view(self):
        return [_p(getattr(self, name)) for name, _, _ in FIELDS]

    def arrays(self):
        return {name: getattr(self, name) for name, _, _ in FIELDS}

    def load(self, arrays):
        for name, dt, w in FIELDS:
            getattr(self, name)[...] = np.asarray(arrays[name], dtype=dt).reshape(self.n, w)

    def copy(self):
        o = OracleState.__new__(OracleState)
        o.n, o.seed, o.env_offset, o.step_counter = self.n, self.seed, self.env_offset, self.step_counter
        for name, _, _ in FIELDS:
            setattr(o, name, getattr(self, name).copy())
        o.counters = self.counters.copy()
        return o

    # -- reference API, batched
    def reset(self, mask=None, random_positions=False):
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        lib().orc_reset(*self._view(), self.n, _p(m), int(bool(random_positions)), self.seed,
                        self.env_offset, self.step_counter)
        self.step_counter += 1

    def move_direction(self, pid, speeds):
        v = np.ascontiguousarray(np.broadcast_to(np.asarray(speeds, np.float64), (self.n,)))
        lib().orc_move_direction(*self._view(), self.n, pid, _p(v), 0.0)

    def move_look(self, pid, angles):
        v = np.ascontiguousarray(np.broadcast_to(np.asarray(angles, np.float64), (self.n,)))
        lib().orc_move_look(*self._view(), self.n, pid, _p(v), 0.0)

    def move_discrete(self, pid, kind, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        lib().orc_move_discrete(*self._view(), self.n, pid, kind, _p(m))

    def shoot(self, pid, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        lib().orc_shoot(*self._view(), self.n, pid, _p(m))

    def game_tick(self):
        lib().orc_game_tick(*self._view(), self.n)

    def projectile_move(self, pid, tick=True, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        lib().orc_projectile_move(*self._view(), self.n, pid, int(bool(tick)), _p(m))

    def check_collision(self):
        h = np.zeros(self.n, np.uint8)
        lib().orc_check_collision(*self._view(), self.n, _p(h))
        return h

    def features(self):
        f = np.zeros((self.n, 2, 18), dtype=np.float64)
        lib().orc_features(*self._view(), self.n, _p(f))
        return f

    def observe(self, reward_kind=0):
        obs = np.zeros((2, self.n, 12), dtype=np.float64)
        rew = np.zeros((2, self.n), dtype=np.float64)
        lib().orc_observe(*self._view(), self.n, _p(obs), _p(rew), reward_kind)
        return obs, rew

    def step(self, actions, tick_limit=2000, auto_reset=False, random_positions=True,
             reward_kind=0, want_obs=True, want_reset_obs=False):
        a = np.ascontiguousarray(actions, dtype=np.float32).reshape(2, self.n, 2)
        obs = np.zeros((2, self.n, 12), np.float64) if want_obs else None
        rew = np.zeros((2, self.n), np.float64) if want_obs else None
        obs_r = np.zeros((2, self.n, 12), np.float64) if want_reset_obs else None
        done = np.zeros(self.n, np.uint8)
        win = np.zeros(self.n, np.uint8)
        lib().orc_step(*self._view(), self.n, _p(a), _p(obs), _p(rew), reward_kind, _p(done), _p(win),
                       int(tick_limit), int(bool(auto_reset)), int(bool(random_positions)), _p(obs_r),
                       self.seed, self.env_offset, self.step_counter, _p(self.counters))
        self.step_counter += 1
        return dict(obs=obs, reward=rew, done=done, winner=win, obs_reset=obs_r)

    def gen_random_actions(self, n_ticks):
        a = np.zeros((n_ticks, 2, self.n, 2), np.float32)
        lib().orc_gen_random_actions(self.n, _p(a), int(n_ticks), self.seed, self.env_offset,
                                     self.step_counter)
        return a

    def rollout_random(self, n_ticks, tick_limit=2000):
        lib().orc_rollout_random(*self._view(), self.n, int(n_ticks), int(tick_limit), self.seed,
                                 self.env_offset, self.step_counter, _p(self.counters))
        self.step_counter += int(n_ticks)


def philox4x32_10(ctr, key):
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.zeros(4, np.uint32)
    lib().orc_philox4x32_10(_p(c), _p(k), _p(out))
    return out


def max_dist():
    return lib().orc_max_dist()
