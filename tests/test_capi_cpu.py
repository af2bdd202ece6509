"""CPU-side checks of the drop-in boundary: libskillshot builds, loads, exports
every symbol include/skillshot.h declares, fails loudly when a GPU is asked
for and absent (no CPU fallback), and serves device = -1 with its CPU
backend."""
import ctypes
import os
import re
import subprocess

import pytest
import torch

import skillshot_learning_amd as ssa
from skillshot_learning_amd import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "skillshot.h")


def header_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sk_[a-z_0-9]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert header_symbols() == sorted(_capi.EXPORTS)


def test_library_exports_every_header_symbol():
    path = _capi.lib_path()
    ssa.load_library()
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (sk_[a-z_0-9]+)$", out, flags=re.M))
    missing = set(header_symbols()) - exported
    assert not missing, missing
    L = ssa.load_library()
    for name in header_symbols():
        assert getattr(L, name) is not None


def test_library_is_gfx950_code_object():
    data = open(_capi.lib_path(), "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in data  # the offload bundle targets gfx950 only
    assert b"--gfx94" not in data and b"--gfx90" not in data


def test_default_config_is_reference():
    c = _capi.default_config()
    # SkillshotGame.py:11,17-18,15 ; Player.py:9-15 ; Projectile.py:5-10
    assert (c.board_w, c.board_h) == (250, 250)
    assert (c.player_size, c.projectile_size) == (5, 3)
    assert (c.player_speed, c.projectile_speed, c.cooldown_max) == (3, 5, 15)
    assert c.look_speed == 0.25
    assert (c.fixed_p1_x, c.fixed_p1_y, c.fixed_p2_x, c.fixed_p2_y) == (50, 50, 200, 200)
    assert (c.rand_lo, c.rand_hi) == (25, 225)


def test_abi_errors_without_device():
    L = ssa.load_library()
    h = ctypes.c_void_p()
    assert L.sk_env_create(ctypes.byref(h), 0, 0, 0, 0, None) == _capi.SK_EINVAL
    assert b"n_envs" in L.sk_last_error()
    assert L.sk_env_destroy(None) == _capi.SK_EINVAL
    assert L.sk_env_step(None, None, None, None, 0, None, None, 0, 0, 0, None, None) == _capi.SK_EINVAL
    if not torch.cuda.is_available():
        rc = L.sk_env_create(ctypes.byref(h), 16, 0, 0, 0, None)
        assert rc == _capi.SK_ENODEV
        assert h.value is None


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure path")
def test_no_cpu_fallback():
    """a GPU request without a GPU fails loudly; the CPU backend is only ever
    the one asked for (device = -1 / "cpu"), never a silent substitute"""
    with pytest.raises(ssa.SkillshotError):
        ssa.VecSkillshotGame(8, device="cuda")
    with pytest.raises(ssa.SkillshotError):
        ssa.VecSkillshotGame(8, device="meta")
    g = ssa.VecSkillshotGame(8, device="cpu")
    assert g.is_cpu and g.pos.device.type == "cpu"


def test_cpu_backend_through_the_abi():
    """sk_env_create(device = -1): engine-owned host state, the fixed start,
    host-pointer calls (device -1 = CPU)"""
    L = ssa.load_library()
    h = ctypes.c_void_p()
    assert L.sk_env_create(ctypes.byref(h), 3, 0, 7, -1, None) == _capi.SK_OK
    v = _capi.SkStateView()
    assert L.sk_env_get_view(h, ctypes.byref(v)) == _capi.SK_OK
    pos = (ctypes.c_int32 * 12).from_address(v.pos)
    assert list(pos[:4]) == [50, 50, 200, 200]  # SkillshotGame.py:17-18
    acts = (ctypes.c_float * 12)(*([0.5, 0.25] * 6))
    done = (ctypes.c_uint8 * 3)()
    assert L.sk_env_step(h, acts, None, None, 0, done, None, 2000, 1, 1, None, None) == _capi.SK_OK
    step = ctypes.c_uint64()
    assert L.sk_env_get_step_counter(h, ctypes.byref(step)) == _capi.SK_OK and step.value == 1
    assert L.sk_env_destroy(h) == _capi.SK_OK


def test_partial_layout_index_is_a_permutation():
    """the gradient-partial layout (csrc/sk_partial.hpp): a permutation of the
    critic's flat parameters that moves W2's action columns behind its
    256-column rows; identity for the actor"""
    import torch
    from skillshot_learning_amd.update_kernel import partial_index
    c = partial_index(36609)
    assert torch.equal(torch.sort(c).values, torch.arange(36609))
    w2 = 256 * 12 + 256
    assert int(c[w2 + 258 + 5]) == w2 + 256 + 5          # W2[1][5]
    assert int(c[w2 + 258 + 257]) == w2 + 128 * 256 + 3  # W2[1][257] (action column 1)
    assert torch.equal(c[:w2], torch.arange(w2)) and torch.equal(c[w2 + 128 * 258:], torch.arange(w2 + 128 * 258, 36609))
    assert torch.equal(partial_index(36482), torch.arange(36482))


@pytest.mark.parametrize("exclude", [-1, 64, 65, 1 << 40])
def test_sampled_critic_rejects_exclude_outside_ring(exclude):
    """sk_ring_sample.exclude outside [0, capacity) is SK_EINVAL in every
    in-launch gather (sk_critic_grad_f32_sampled, sk_critic_grad_bootstrap_
    sampled), as in sk_replay_sample_excl: a negative draw window would index
    outside the ring.  The checks run before any launch, so the
    dummy (aligned, never dereferenced) pointers are safe without a GPU."""
    from skillshot_learning_amd.update_kernel import RingSample
    L = ssa.load_library()
    fake = ctypes.c_void_p(0x1000)
    q = RingSample(0x1000, 64, 0x1000, 0, 0, 0x1000, 0x1000, 0x1000, 0x1000, 0x1000, exclude)
    rc = L.sk_critic_grad_f32_sampled(fake, ctypes.byref(q), 0.0, None, None, 16, 0, 1.0, 0, fake, fake, None, 0,
                                      None, None, fake, None)
    assert rc == _capi.SK_EINVAL
    rc = L.sk_critic_grad_bootstrap_sampled(fake, ctypes.byref(q), 0.0, None, None, 16, 0, 1.0, 0, fake, fake, None,
                                            0, None, None, None)
    assert rc == _capi.SK_EINVAL
    assert L.sk_replay_sample_excl(fake, 64, fake, 0, 0, 16, fake, fake, fake, fake, fake, exclude,
                                   None) == _capi.SK_EINVAL


def test_gpu_only_entry_points_refuse_the_cpu_backend():
    """sk_env_act_step / sk_env_act_episode are GPU-only (the fused actor):
    on a CPU-backend handle they return SK_EINVAL, never run a host
    substitute; sk_actor_split_pack_bytes reports the split pack's size"""
    L = ssa.load_library()
    h = ctypes.c_void_p()
    assert L.sk_env_create(ctypes.byref(h), 8, 0, 7, -1, None) == _capi.SK_OK
    buf = (ctypes.c_float * 4096)()
    ln = (ctypes.c_int32 * 8)()
    rc = L.sk_env_act_episode(h, buf, buf, buf, buf, buf, ln, 10, 0.5, 0.0, 1, None, 0, 2000, None)
    assert rc == _capi.SK_EINVAL and b"GPU" in L.sk_last_error()
    assert L.sk_env_destroy(h) == _capi.SK_OK
    assert L.sk_actor_split_pack_bytes() == 4 * (8 * 64 * 8 + 4 * 16 * 64 * 8) * 2


def test_resident_fit_rejects_bad_arguments():
    """sk_fit_critic_f32 / sk_fit_actor_f32 (ABI 11, models_fit's resident
    passes) check their arguments before any launch: missing buffers, no
    minibatch, a step-counter count outside [1, 64] or an exchange buffer off
    its 16-byte alignment are SK_EINVAL (the dummy pointers are never
    dereferenced, so no GPU is needed); the exchange buffer's size is fixed"""
    L = ssa.load_library()
    f = ctypes.c_void_p(0x1000)
    off = ctypes.c_void_p(0x1008)
    assert L.sk_fit_xbuf_bytes() == 65536 * 8

    def critic(xbuf=f, n=4, n_steps=1, targets=f):
        return L.sk_fit_critic_f32(f, f, f, f, n_steps, f, f, targets, n, 0, f, 1e-3, 0.9, 0.999, 1e-7, xbuf, f, f,
                                   None, None)

    def actor(xbuf=f, n=4, n_steps=1, zbuf=f):
        return L.sk_fit_actor_f32(f, f, f, f, n_steps, f, f, n, 1e-3, 0.9, 0.999, 1e-7, xbuf, f, f, zbuf, None)

    for rc in (critic(n=0), critic(n_steps=0), critic(n_steps=65), critic(xbuf=None), critic(xbuf=off),
               critic(targets=None), actor(n=0), actor(n_steps=0), actor(xbuf=off), actor(zbuf=None)):
        assert rc == _capi.SK_EINVAL
