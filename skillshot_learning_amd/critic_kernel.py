"""Fused MFMA critic forward and DDPG bootstrap target (csrc/sk_critic.hip)
bound to torch Actor/Critic modules.

The torch modules stay the master copies; `refresh()` repacks their weights
into the kernels' fragment layouts on device (one small kernel per net).
"""
import ctypes

import torch

from . import _capi
from ._capi import SkillshotError


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


class CriticKernel:
    """Q(s, a) of a Critic at inference (Dropout off), one launch."""

    def __init__(self, critic):
        self.critic = critic
        self.L = _capi.load()
        p = next(critic.parameters())
        if p.device.type != "cuda":
            raise SkillshotError("CriticKernel needs the critic on a gfx950 GPU")
        self.device = p.device
        self.buf = torch.empty(int(self.L.sk_critic_packed_bytes()), dtype=torch.uint8, device=self.device)
        self.refresh()

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    @torch.no_grad()
    def refresh(self):
        c = self.critic
        ws = [t.detach().contiguous() for t in (c.l1.weight, c.l1.bias, c.l2.weight, c.l2.bias, c.l3.weight,
                                                c.l3.bias)]
        self._keep = ws
        rc = self.L.sk_critic_pack(*[_p(t) for t in ws], _p(self.buf), self._stream())
        if rc != 0:
            raise SkillshotError(f"sk_critic_pack failed ({rc})")

    @torch.no_grad()
    def __call__(self, obs, actions, out=None):
        """obs float32 [M, 12], actions float32 [M, 2] -> q float32 [M]."""
        x, a = obs.float().contiguous(), actions.float().contiguous()
        if x.dim() != 2 or x.shape[1] != 12 or a.shape != (x.shape[0], 2):
            raise ValueError("obs must be [M, 12] and actions [M, 2]")
        q = out if out is not None else torch.empty(x.shape[0], dtype=torch.float32, device=self.device)
        rc = self.L.sk_critic_forward(_p(self.buf), _p(x), _p(a), _p(q), x.shape[0], self._stream())
        if rc != 0:
            raise SkillshotError(f"sk_critic_forward failed ({rc})")
        return q


class TargetQKernel:
    """Q'(s, mu'(s)) of an (actor, critic) pair in one launch: the DDPG
    bootstrap term.  `refresh()` after every change of either net."""

    def __init__(self, actor, critic):
        from .actor_kernel import ActorKernel
        self.actor_k = ActorKernel(actor)
        self.critic_k = CriticKernel(critic)
        self.L = self.critic_k.L
        self.device = self.critic_k.device

    def refresh(self):
        self.actor_k.refresh()
        self.critic_k.refresh()

    @torch.no_grad()
    def __call__(self, obs, out=None, actions_out=None):
        x = obs.float().contiguous()
        if x.dim() != 2 or x.shape[1] != 12:
            raise ValueError("obs must be [M, 12]")
        q = out if out is not None else torch.empty(x.shape[0], dtype=torch.float32, device=self.device)
        rc = self.L.sk_target_q(_p(self.actor_k.buf), _p(self.critic_k.buf), _p(x), _p(q),
                                None if actions_out is None else _p(actions_out), x.shape[0],
                                self.critic_k._stream())
        if rc != 0:
            raise SkillshotError(f"sk_target_q failed ({rc})")
        return q

    @torch.no_grad()
    def target(self, next_obs, reward, done, gamma, out=None):
        """y = r + gamma (1 - done) Q'(s', mu'(s')) in the same launch."""
        x = next_obs.float().contiguous()
        r, d = reward.float().contiguous(), done.float().contiguous()
        y = out if out is not None else torch.empty(x.shape[0], dtype=torch.float32, device=self.device)
        rc = self.L.sk_target_y(_p(self.actor_k.buf), _p(self.critic_k.buf), _p(x), _p(r), _p(d), float(gamma),
                                _p(y), x.shape[0], self.critic_k._stream())
        if rc != 0:
            raise SkillshotError(f"sk_target_y failed ({rc})")
        return y
