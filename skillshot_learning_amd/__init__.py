"""skillshot_learning_amd — MI355X-native batched Skillshot self-play engine.

Drop-in for the per-tick step path of adrientremblay/Skillshot_Learning:
the game core (SkillshotGame/Player/Projectile) and the learner's per-tick
observation/reward protocol run as hand-written gfx950 HIP kernels in
libskillshot.so (C ABI: include/skillshot.h), bound here with ctypes.
"""
from ._capi import SkillshotError, load as load_library, lib_path  # noqa: F401
from .vec_env import FEATURE_KEYS, VecSkillshotGame  # noqa: F401

__all__ = ["SkillshotError", "VecSkillshotGame", "FEATURE_KEYS", "load_library", "lib_path"]
