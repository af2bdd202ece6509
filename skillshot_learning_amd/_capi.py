"""ctypes binding of libskillshot (include/skillshot.h).

torch is imported before the library is loaded so that libskillshot resolves
libamdhip64.so.7 to the HIP runtime torch already loaded: one runtime per
process, torch's stream handles valid for our launches.

There is no CPU fallback: if the library is missing or no gfx950 device is
present, calls raise SkillshotError.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

from . import build as _build

SK_OK, SK_EINVAL, SK_EHIP, SK_ENOMEM, SK_ENODEV = 0, -1, -2, -3, -4
SK_REWARD_LOOKING, SK_REWARD_SIMPLE = 0, 1
ABI_VERSION = 11

# every symbol include/skillshot.h declares
EXPORTS = (
    "sk_last_error", "sk_abi_version", "sk_config_default", "sk_env_create", "sk_env_attach",
    "sk_env_destroy", "sk_env_get_view", "sk_env_counters_ptr", "sk_env_counter_slots", "sk_env_read_counters",
    "sk_env_clear_counters", "sk_env_get_step_counter",
    "sk_env_set_step_counter", "sk_env_sync_step_counter", "sk_env_reset", "sk_player_move_direction", "sk_player_move_look",
    "sk_player_move_discrete", "sk_player_shoot", "sk_projectile_move", "sk_game_check_collision", "sk_game_tick", "sk_env_features", "sk_env_observe",
    "sk_env_step", "sk_env_step_insert", "sk_env_act_step", "sk_env_act_step_job", "sk_env_act_episode", "sk_env_step_multi", "sk_env_step_multi_obs", "sk_gen_random_actions", "sk_env_rollout_random",
    "sk_actor_packed_bytes", "sk_actor_pack", "sk_actor_forward", "sk_actor_forward_dev",
    "sk_actor_forward_advance", "sk_actor_forward_noise",
    "sk_critic_packed_bytes", "sk_critic_pack", "sk_critic_forward", "sk_target_q",
    "sk_grad_packed_bytes", "sk_update_partials", "sk_grad_pack", "sk_critic_grad", "sk_actor_grad", "sk_adam_flat",
    "sk_adam_flat_packed", "sk_adam_flat_sliced", "sk_update_scratch_f32",
    "sk_target_y", "sk_replay_insert", "sk_replay_sample", "sk_replay_insert_sample", "sk_grad_pack_flat",
    "sk_critic_grad_bootstrap",
    "sk_update_partials_f32", "sk_actor_forward_f32", "sk_actor_split_pack_bytes", "sk_actor_split_pack_f32", "sk_critic_grad_f32", "sk_critic_grad_f32_sampled",
    "sk_critic_grad_bootstrap_sampled", "sk_actor_grad_f32", "sk_actor_grad_f32_step",
    "sk_critic_grad_f32_sampled_step", "sk_critic_grad_f32_step", "sk_replay_sample_excl",
    "sk_fit_xbuf_bytes", "sk_fit_critic_f32", "sk_fit_actor_f32",
)


class SkillshotError(RuntimeError):
    pass


class SkConfig(ctypes.Structure):
    _fields_ = [("board_w", ctypes.c_int32), ("board_h", ctypes.c_int32),
                ("player_size", ctypes.c_int32), ("projectile_size", ctypes.c_int32),
                ("player_speed", ctypes.c_int32), ("projectile_speed", ctypes.c_int32),
                ("cooldown_max", ctypes.c_int32), ("look_speed", ctypes.c_double),
                ("fixed_p1_x", ctypes.c_int32), ("fixed_p1_y", ctypes.c_int32),
                ("fixed_p2_x", ctypes.c_int32), ("fixed_p2_y", ctypes.c_int32),
                ("rand_lo", ctypes.c_int32), ("rand_hi", ctypes.c_int32)]


class SkStateView(ctypes.Structure):
    _fields_ = [("n_envs", ctypes.c_int32), ("pos", ctypes.c_void_p), ("rot", ctypes.c_void_p),
                ("qpos", ctypes.c_void_p), ("qrot", ctypes.c_void_p), ("qcdage", ctypes.c_void_p),
                ("misc", ctypes.c_void_p)]


class SkStepJob(ctypes.Structure):
    """sk_step_job: one prepared acting launch (opaque)"""
    _fields_ = [("opaque", ctypes.c_uint64 * 128)]


class SkCounters(ctypes.Structure):
    _fields_ = [("dones", ctypes.c_uint64), ("hits_p1", ctypes.c_uint64), ("hits_p2", ctypes.c_uint64),
                ("ticks_sum", ctypes.c_uint64)]


_lib = None


def lib_path():
    return _build.LIB_PATH


def load(build_if_missing=True):
    """Load libskillshot (building it in-tree first if it is absent/stale)."""
    global _lib
    if _lib is not None:
        return _lib
    path = _build.LIB_PATH
    if build_if_missing and (not os.path.exists(path) or _build.needs_build()):
        _build.build()
    if not os.path.exists(path):
        raise SkillshotError(f"libskillshot not built ({path}); run python -m skillshot_learning_amd.build")
    L = ctypes.CDLL(path)
    P, i32, i64, u64, f64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
    f32 = ctypes.c_float
    PP = ctypes.POINTER(ctypes.c_void_p)
    sig = {
        "sk_last_error": ([], ctypes.c_char_p),
        "sk_abi_version": ([], ctypes.c_int),
        "sk_config_default": ([ctypes.POINTER(SkConfig)], None),
        "sk_env_create": ([PP, i32, i64, u64, i32, ctypes.POINTER(SkConfig)], ctypes.c_int),
        "sk_env_attach": ([PP, ctypes.POINTER(SkStateView), i64, u64, i32, ctypes.POINTER(SkConfig)],
                          ctypes.c_int),
        "sk_env_destroy": ([P], ctypes.c_int),
        "sk_env_get_view": ([P, ctypes.POINTER(SkStateView)], ctypes.c_int),
        "sk_env_counters_ptr": ([P, PP], ctypes.c_int),
        "sk_env_counter_slots": ([P, ctypes.POINTER(ctypes.c_int64)], ctypes.c_int),
        "sk_env_read_counters": ([P, ctypes.POINTER(SkCounters), P], ctypes.c_int),
        "sk_env_clear_counters": ([P, P], ctypes.c_int),
        "sk_env_get_step_counter": ([P, ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
        "sk_env_set_step_counter": ([P, u64], ctypes.c_int),
        "sk_env_sync_step_counter": ([P, P], ctypes.c_int),
        "sk_env_reset": ([P, P, i32, P], ctypes.c_int),
        "sk_player_move_direction": ([P, i32, P, f64, P], ctypes.c_int),
        "sk_player_move_look": ([P, i32, P, f64, P], ctypes.c_int),
        "sk_player_move_discrete": ([P, i32, i32, P, P], ctypes.c_int),
        "sk_player_shoot": ([P, i32, P, P], ctypes.c_int),
        "sk_projectile_move": ([P, i32, i32, P, P], ctypes.c_int),
        "sk_game_check_collision": ([P, P, P], ctypes.c_int),
        "sk_game_tick": ([P, P], ctypes.c_int),
        "sk_env_features": ([P, P, P], ctypes.c_int),
        "sk_env_observe": ([P, P, P, i32, P], ctypes.c_int),
        "sk_env_step": ([P, P, P, P, i32, P, P, i32, i32, i32, P, P], ctypes.c_int),
        "sk_env_step_insert": ([P, P, P, P, i32, P, P, i32, i32, i32, P, P, P, i64, P, P, P, P], ctypes.c_int),
        "sk_env_act_step": ([P, P, P, P, P, f32, f32, u64, P, P, P, i32, P, P, i32, i32, i32, P, P, i64, P, P, P, P],
                            ctypes.c_int),
        "sk_env_act_episode": ([P, P, P, P, P, P, P, i32, f32, f32, u64, P, i32, i32, P], ctypes.c_int),
        "sk_env_act_step_job": ([P, P, P, P, P, f32, f32, u64, P, P, P, i32, P, P, i32, i32, i32, P, P, i64, P, P, P,
                                 ctypes.POINTER(SkStepJob)], ctypes.c_int),
        "sk_env_step_multi": ([P, P, i64, i64, i32, P, P, i64, i32, i32, i32, P], ctypes.c_int),
        "sk_env_step_multi_obs": ([P, P, i64, i64, i32, P, P, i32, P, P, i64, i64, i32, i32, i32, P], ctypes.c_int),
        "sk_gen_random_actions": ([P, P, i32, P], ctypes.c_int),
        "sk_env_rollout_random": ([P, i32, i32, P], ctypes.c_int),
        "sk_actor_packed_bytes": ([], ctypes.c_size_t),
        "sk_actor_pack": ([P, P, P, P, P, P, P, P], ctypes.c_int),
        "sk_actor_forward": ([P, P, P, i64, ctypes.c_float, u64, u64, P], ctypes.c_int),
        "sk_actor_forward_dev": ([P, P, P, i64, ctypes.c_float, u64, P, P], ctypes.c_int),
        "sk_actor_forward_advance": ([P, P, P, i64, ctypes.c_float, u64, P, P], ctypes.c_int),
        "sk_actor_forward_noise": ([P, P, P, i64, ctypes.c_float, ctypes.c_float, u64, P, P], ctypes.c_int),
        "sk_critic_packed_bytes": ([], ctypes.c_size_t),
        "sk_critic_pack": ([P, P, P, P, P, P, P, P], ctypes.c_int),
        "sk_critic_forward": ([P, P, P, P, i64, P], ctypes.c_int),
        "sk_target_q": ([P, P, P, P, P, i64, P], ctypes.c_int),
        "sk_grad_packed_bytes": ([], ctypes.c_size_t),
        "sk_update_partials": ([i64], ctypes.c_int64),
        "sk_grad_pack": ([P, P, P, i32, P, P, P, i32, P, P], ctypes.c_int),
        "sk_critic_grad": ([P, P, P, P, i64, i64, f32, u64, P, P, P, i32, P, P, P], ctypes.c_int),
        "sk_actor_grad": ([P, P, P, i64, f32, P, P, i32, P, P], ctypes.c_int),
        "sk_adam_flat_packed": ([P, i32, i32, P, P, i32, P, P, P, P, f32, f32, f32, f32, P, f32, P, f32, P, P, P, P],
                                ctypes.c_int),
        "sk_adam_flat": ([P, i32, i32, P, P, i32, P, P, P, P, f32, f32, f32, f32, P, f32, P, f32, P, P, P],
                         ctypes.c_int),
        "sk_target_y": ([P, P, P, P, P, f32, P, i64, P], ctypes.c_int),
        "sk_replay_insert": ([P, i64, P, P, P, P, P, P, P, i64, i64, P], ctypes.c_int),
        "sk_replay_sample": ([P, i64, P, u64, i32, i64, P, P, P, P, P, P], ctypes.c_int),
        "sk_replay_sample_excl": ([P, i64, P, u64, i32, i64, P, P, P, P, P, i64, P], ctypes.c_int),
        "sk_replay_insert_sample": ([P, i64, P, P, P, P, P, P, P, i64, i64, u64, i32, i64, P, P, P, P, P, P],
                                    ctypes.c_int),
        "sk_grad_pack_flat": ([P, P, P, P, i32, P], ctypes.c_int),
        "sk_critic_grad_bootstrap": ([P, P, P, P, P, P, P, f32, P, P, i64, i64, f32, u64, P, P, P, i32, P, P, P],
                                     ctypes.c_int),
        "sk_update_partials_f32": ([i64], ctypes.c_int64),
        "sk_actor_forward_f32": ([P, P, P, P, i64, f32, f32, u64, P, P], ctypes.c_int),
        "sk_actor_split_pack_bytes": ([], ctypes.c_size_t),
        "sk_actor_split_pack_f32": ([P, P, P], ctypes.c_int),
        "sk_critic_grad_f32": ([P, P, P, P, P, P, P, f32, P, P, i64, i64, f32, u64, P, P, P, i32, P, P, P, P],
                               ctypes.c_int),
        "sk_critic_grad_f32_sampled": ([P, P, f32, P, P, i64, i64, f32, u64, P, P, P, i32, P, P, P, P],
                                       ctypes.c_int),
        "sk_critic_grad_f32_step": ([P, P, P, P, P, P, P, f32, P, P, i64, i64, f32, u64, P, P, P, i32, P, P, P,
                                     ctypes.POINTER(SkStepJob), P], ctypes.c_int),
        "sk_critic_grad_f32_sampled_step": ([P, P, f32, P, P, i64, i64, f32, u64, P, P, P, i32, P, P, P,
                                             ctypes.POINTER(SkStepJob), P], ctypes.c_int),
        "sk_critic_grad_bootstrap_sampled": ([P, P, f32, P, P, i64, i64, f32, u64, P, P, P, i32, P, P, P],
                                             ctypes.c_int),
        "sk_actor_grad_f32": ([P, P, P, i64, f32, P, P, i32, P, P, P], ctypes.c_int),
        "sk_actor_grad_f32_step": ([P, P, P, i64, f32, P, P, i32, P, P, ctypes.POINTER(SkStepJob), P], ctypes.c_int),
        "sk_update_scratch_f32": ([i64, P], ctypes.c_int64),
        "sk_adam_flat_sliced": ([P, i32, P, i32, i32, P, P, i32, P, P, P, P, f32, f32, f32, f32, P, f32, P, f32, P, P,
                                 P, P], ctypes.c_int),
        "sk_fit_xbuf_bytes": ([], ctypes.c_size_t),
        "sk_fit_critic_f32": ([P, P, P, P, i32, P, P, P, i32, u64, P, f32, f32, f32, f32, P, P, P, P, P], ctypes.c_int),
        "sk_fit_actor_f32": ([P, P, P, P, i32, P, P, i32, f32, f32, f32, f32, P, P, P, P, P], ctypes.c_int),
    }
    for name, (argt, rest) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = argt
        fn.restype = rest
    if L.sk_abi_version() != ABI_VERSION:
        raise SkillshotError(f"libskillshot ABI {L.sk_abi_version()} != expected {ABI_VERSION}")
    _lib = L
    return L


def check(rc):
    if rc != SK_OK:
        msg = _lib.sk_last_error().decode(errors="replace") if _lib is not None else ""
        raise SkillshotError(f"libskillshot error {rc}: {msg}")
    return rc


def default_config():
    c = SkConfig()
    load().sk_config_default(ctypes.byref(c))
    return c
