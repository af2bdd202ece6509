"""Fused MFMA actor forward (csrc/sk_actor.hip) bound to a torch Actor.

The torch module stays the master copy (fp32, trained by autograd); after each
optimiser step `refresh()` repacks its weights into the kernel's bf16 MFMA
fragment layout on device (one small kernel, no host copy) — unless the
fused update's Adam launch writes that pack itself.  The noise call number
lives on device and each noisy launch advances it (sk_actor_forward_advance),
so a captured hipGraph of the learner tick draws fresh parameter noise on
every replay with no extra launch.
"""
import ctypes

import torch

from . import _capi
from ._capi import SkillshotError


class ActorKernel:
    def __init__(self, actor, seed=0):
        self.actor = actor
        self.L = _capi.load()
        p = next(actor.parameters())
        if p.device.type != "cuda":
            raise SkillshotError("ActorKernel needs the actor on a gfx950 GPU")
        self.device = p.device
        self.buf = torch.empty(int(self.L.sk_actor_packed_bytes()), dtype=torch.uint8, device=self.device)
        self.seed = int(seed) & ((1 << 64) - 1)
        # device noise-call number, the launch's arrival slot and its 8 group
        # slots (sk_actor_forward_noise: SK_ACTOR_COUNTER_WORDS words)
        self._ctr = torch.zeros(130, dtype=torch.int64, device=self.device)
        self.counter = self._ctr[:1]
        self.refresh()

    @property
    def calls(self):
        """the device's noise call number (the draws so far; a host sync).
        No host mirror is kept: launches that draw advance it on device, an
        episode launch by the ticks it played"""
        return int(self._ctr[0].item())

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    @torch.no_grad()
    def refresh(self):
        a = self.actor
        ws = [t.detach().contiguous() for t in (a.l1.weight, a.l1.bias, a.l2.weight, a.l2.bias, a.l3.weight,
                                                a.l3.bias)]
        self._keep = ws
        rc = self.L.sk_actor_pack(*[ctypes.c_void_p(t.data_ptr()) for t in ws], ctypes.c_void_p(self.buf.data_ptr()),
                                  self._stream())
        if rc != 0:
            raise SkillshotError(f"sk_actor_pack failed ({rc})")

    fused_action_noise = True  # model_act_action_noise's N(0, sd) is drawn in the kernel (sk_actor_forward_noise)

    @torch.no_grad()
    def __call__(self, obs, noise_sd=0.0, generator=None, out=None, action_sd=0.0):
        """obs float32 [M, 12] -> actions float32 [M, 2]; noise_sd: parameter
        noise, action_sd: action noise on the tanh outputs."""
        x = obs if obs.dtype == torch.float32 else obs.float()
        x = x.contiguous()
        if x.dim() != 2 or x.shape[1] != 12:
            raise ValueError("obs must be [M, 12]")
        m = x.shape[0]
        y = out if out is not None else torch.empty((m, 2), dtype=torch.float32, device=self.device)
        rc = self.L.sk_actor_forward_noise(ctypes.c_void_p(self.buf.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                           ctypes.c_void_p(y.data_ptr()), m, float(noise_sd), float(action_sd),
                                           self.seed, ctypes.c_void_p(self._ctr.data_ptr()), self._stream())
        if rc != 0:
            raise SkillshotError(f"sk_actor_forward failed ({rc})")
        return y


class ActorKernel32:
    """The actor forward at the reference's precision (csrc/sk_learn32.hip
    k_actor_fwd32 / k_actor_fwd16), reading biases and W3 from the actor's
    flat fp32 parameter vector and W1 / W2 from its split pack (`pack`,
    sk_split.hpp: three bf16 pieces per weight, so the 32-row tile computes
    fp32 products at the bf16 MFMA rate).  The pack follows the parameters:
    the fused update's Adam launch rewrites it (DDPG._fused.split_pack), and
    a change made through torch (optimizer steps, load_state_dict, copy_)
    bumps the parameters' version counters, on which every call repacks
    (ensure_pack; the parameters are views of the flat buffer through
    `.data`, so each keeps its own counter).  Same call interface as
    ActorKernel."""

    buf = None  # no bf16 forward pack

    def __init__(self, actor, seed=0):
        from .update_kernel import flatten_module
        self.actor = actor
        self.L = _capi.load()
        p = next(actor.parameters())
        if p.device.type != "cuda":
            raise SkillshotError("ActorKernel32 needs the actor on a gfx950 GPU")
        self.device = p.device
        self.flat = flatten_module(actor)
        self.seed = int(seed) & ((1 << 64) - 1)
        self._ctr = torch.zeros(130, dtype=torch.int64, device=self.device)  # SK_ACTOR_COUNTER_WORDS
        self.counter = self._ctr[:1]
        self.pack = torch.zeros(int(self.L.sk_actor_split_pack_bytes()), dtype=torch.uint8, device=self.device)
        self._packed = None  # (flat buffer, the parameters' versions) the pack was last written from
        self.ensure_pack()

    @property
    def calls(self):
        """the device's noise call number (the draws so far; a host sync).
        No host mirror is kept: launches that draw advance it on device, an
        episode launch by the ticks it played"""
        return int(self._ctr[0].item())

    def refresh(self):
        """repack from the current flat parameters"""
        from .update_kernel import flatten_module
        self.flat = flatten_module(self.actor)  # idempotent: the parameters stay views of it
        rc = self.L.sk_actor_split_pack_f32(ctypes.c_void_p(self.flat.data_ptr()),
                                            ctypes.c_void_p(self.pack.data_ptr()), self._stream())
        if rc != 0:
            raise SkillshotError(f"sk_actor_split_pack_f32 failed ({rc})")
        self._packed = self._key()

    def ensure_pack(self):
        """the split pack, repacked first if the parameters were changed
        through torch since it was written (returns it)"""
        if self._packed != self._key():
            self.refresh()
        return self.pack

    def _key(self):
        return (self.flat.data_ptr(),) + tuple(p._version for p in self.actor.parameters())

    fused_action_noise = True  # model_act_action_noise's N(0, sd) is drawn in the kernel
    fused_act_step = True  # the self-play tick runs it inside the step launch (VecSkillshotGame.act_step)

    @torch.no_grad()
    def __call__(self, obs, noise_sd=0.0, generator=None, out=None, action_sd=0.0):
        """obs float32 [M, 12] -> actions float32 [M, 2]; noise_sd: parameter
        noise, action_sd: action noise on the tanh outputs."""
        x = obs if obs.dtype == torch.float32 else obs.float()
        x = x.contiguous()
        if x.dim() != 2 or x.shape[1] != 12:
            raise ValueError("obs must be [M, 12]")
        m = x.shape[0]
        y = out if out is not None else torch.empty((m, 2), dtype=torch.float32, device=self.device)
        pack = self.ensure_pack()
        rc = self.L.sk_actor_forward_f32(ctypes.c_void_p(self.flat.data_ptr()), ctypes.c_void_p(pack.data_ptr()),
                                         ctypes.c_void_p(x.data_ptr()),
                                         ctypes.c_void_p(y.data_ptr()), m, float(noise_sd), float(action_sd),
                                         self.seed, ctypes.c_void_p(self._ctr.data_ptr()), self._stream())
        if rc != 0:
            raise SkillshotError(f"sk_actor_forward_f32 failed ({rc})")
        return y

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
