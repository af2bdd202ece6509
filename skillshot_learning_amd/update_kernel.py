"""The DDPG update on MFMA (csrc/sk_update.hip) bound to the torch nets of a
`learner.DDPG`.

Per update and net: one gradient launch (forward + backward over the whole
minibatch, per-workgroup weight-gradient partials) and one Adam launch (sum
of the partials, torch Adam, soft target update); the weight packs the
gradient kernels read are refreshed after each step.  This replaces the
~100 small torch kernels of `DDPG.critic_step` / `model_actor_fit_step` /
`soft_update` (SkillshotLearner.py:386-443 rule).

The torch modules stay the model: their parameters are rebound as views of
one flat fp32 buffer per net (`.data` swap, so optimiser and state-dict
references stay valid), and the torch Adam state (`exp_avg`, `exp_avg_sq`,
`step`) is rebound as views of flat buffers too, so the kernel path and the
torch path step the same numbers and `state_dict()` sees the kernel's Adam
moments.  Multi-rank: the gradient is written flat, all-reduced (mean) over
RCCL, then applied (two Adam launches).
"""
import contextlib
import ctypes

import torch
import torch.distributed as dist

from . import _capi
from ._capi import SkillshotError


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class RingSample(ctypes.Structure):
    """sk_ring_sample (include/skillshot.h): a minibatch drawn from the replay
    ring inside the critic step (sk_critic_grad_f32_sampled)."""
    _fields_ = [("ring", ctypes.c_void_p), ("capacity", ctypes.c_int64), ("total", ctypes.c_void_p),
                ("seed", ctypes.c_uint64), ("draw", ctypes.c_int32), ("s", ctypes.c_void_p),
                ("a", ctypes.c_void_p), ("r", ctypes.c_void_p), ("s2", ctypes.c_void_p), ("d", ctypes.c_void_p),
                ("exclude", ctypes.c_int64)]


class PackTargets(ctypes.Structure):
    """sk_pack_targets (include/skillshot.h): the packed copies an Adam launch writes."""
    _fields_ = [("param_gpack", ctypes.c_void_p), ("target_gpack", ctypes.c_void_p),
                ("actor_fwd_pack", ctypes.c_void_p), ("ld2", ctypes.c_int32), ("n_out", ctypes.c_int32),
                ("actor_split_pack", ctypes.c_void_p)]


def flatten_module(module):
    """Rebind every parameter of `module` as a view of one flat fp32 buffer
    (idempotent); returns the buffer."""
    flat = getattr(module, "_sk_flat", None)
    params = list(module.parameters())
    if flat is not None and all(p.data.data_ptr() == flat[o:o + p.numel()].data_ptr()
                                for p, o in zip(params, _offsets(params))):
        return flat
    n = sum(p.numel() for p in params)
    flat = torch.empty(n, dtype=torch.float32, device=params[0].device)
    off = 0
    for p in params:
        k = p.numel()
        flat[off:off + k].copy_(p.data.reshape(-1))
        p.data = flat[off:off + k].view_as(p)
        off += k
    module._sk_flat = flat
    return flat


def partial_index(n_params, device=None):
    """Offset of each flat parameter in a gradient-partial row (the layout the
    gradient kernels write and sk_adam_flat sums; csrc/sk_partial.hpp): flat
    order, except the critic's (36,609 parameters) W2 [128][258] as [128][256]
    main columns followed by its [128][2] action columns."""
    idx = torch.arange(n_params, dtype=torch.int64, device=device)
    if n_params != 36609:
        return idx
    w2 = 256 * 12 + 256
    q = idx[w2:w2 + 128 * 258] - w2
    o, i = q // 258, q % 258
    idx[w2:w2 + 128 * 258] = torch.where(i < 256, w2 + o * 256 + i, w2 + 128 * 256 + 2 * o + (i - 256))
    return idx


def _offsets(params):
    out, off = [], 0
    for p in params:
        out.append(off)
        off += p.numel()
    return out


class _AdamState:
    """Adam state (learner.KerasAdam) of one net as flat buffers (views
    rebound into the optimiser's per-parameter state)."""

    def __init__(self, opt, module, flat):
        params = list(module.parameters())
        dev = flat.device
        self.m = torch.zeros_like(flat)
        self.v = torch.zeros_like(flat)
        self.steps = torch.zeros(len(params), dtype=torch.float32, device=dev)
        g = opt.param_groups[0]
        self.lr, (self.b1, self.b2), self.eps = float(g["lr"]), g["betas"], float(g["eps"])
        self.bind(opt, module)

    @torch.no_grad()
    def bind(self, opt, module):
        """copy whatever state the optimiser holds (e.g. just loaded by
        Optimizer.load_state_dict) into the flat buffers, then make the
        optimiser's state views of them again"""
        params = list(module.parameters())
        for i, (p, off) in enumerate(zip(params, _offsets(params))):
            k = p.numel()
            st = opt.state[p]
            if "exp_avg" in st:
                self.m[off:off + k].copy_(st["exp_avg"].reshape(-1))
                self.v[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                self.steps[i].copy_(torch.as_tensor(st["step"], dtype=torch.float32))
            st["exp_avg"] = self.m[off:off + k].view_as(p)
            st["exp_avg_sq"] = self.v[off:off + k].view_as(p)
            st["step"] = self.steps[i]


class _Partials:
    """Gradient partials of one (batch, net): rows [G][n_params] and, for the
    sliced fp32 kernels (sk_update_scratch_f32 > 0), their scratch, whose first
    w1_rows x 3,328 floats are the W1 / b1 contribution rows"""

    def __init__(self, main, scratch=None, w1_rows=0):
        self.main, self.scratch, self.w1_rows = main, scratch, int(w1_rows)

    @property
    def rows(self):
        return self.main.shape[0]


class FusedUpdate:
    """Kernel path of DDPG.critic_step / model_actor_fit_step (+ soft update)."""

    LOSS_HIST = 1024

    def __init__(self, ddpg):
        self.d = ddpg
        self.L = _capi.load()
        dev = ddpg.device
        if dev.type != "cuda":
            raise SkillshotError("FusedUpdate needs the nets on a gfx950 GPU")
        self.dev = dev
        self.fa = flatten_module(ddpg.model_actor)
        self.fc = flatten_module(ddpg.model_critic)
        self.ta = flatten_module(ddpg.target_actor) if ddpg.tau is not None else None
        self.tc = flatten_module(ddpg.target_critic) if ddpg.tau is not None else None
        # fp32: the kernels of csrc/sk_learn32.hip read the flat parameter
        # vectors themselves (no packs); bf16: sk_update.hip's MFMA packs
        self.f32 = getattr(ddpg, "precision", "bf16") == "fp32"
        self.sa = _AdamState(ddpg.optimiser, ddpg.model_actor, self.fa)
        self.sc = _AdamState(ddpg.critic_optimiser, ddpg.model_critic, self.fc)
        # models_fit (the reference rule) has no target nets: it clears this
        self.soft_update_in_adam = True
        nb = int(self.L.sk_grad_packed_bytes())
        self.gpa = torch.empty(nb, dtype=torch.uint8, device=dev)
        self.gpc = torch.empty(nb, dtype=torch.uint8, device=dev)
        # target nets' packs (the bootstrap target inside the critic step)
        self.gpta = torch.empty(nb, dtype=torch.uint8, device=dev) if self.ta is not None else self.gpa
        self.gptc = torch.empty(nb, dtype=torch.uint8, device=dev) if self.tc is not None else self.gpc
        # Dropout key and call number: the DDPG's (shared with the torch
        # path; masks keyed by global batch row).  Loss accumulators [sum
        # (q-y)^2, sum Q] on device; the Adam launch advances the call number,
        # reads-and-clears the accumulators and writes the step's loss into a
        # history slot (the returned device scalar stays valid for LOSS_HIST
        # further steps)
        self.seed = ddpg.drop_seed
        self.calls = ddpg.drop_calls
        self.stats = torch.zeros(2, dtype=torch.float32, device=dev)
        self.loss_hist = torch.zeros(2, self.LOSS_HIST, dtype=torch.float32, device=dev)
        self._li = [0, 0]
        self._loss_private = None
        self._partials = {}
        self.grad_flat = None
        # the actor forward kernel's weight pack (ActorKernel.buf), written by
        # the actor's Adam launch when bound (SkillshotLearner binds it)
        self.fwd_pack = None
        # the fp32 actor's split pack (ActorKernel32.pack, sk_split.hpp),
        # likewise written by the actor's Adam launch when bound
        self.split_pack = None
        self.pack()

    def rebind_optimisers(self):
        """after the optimisers' state was replaced (load_state_dict): the
        loaded moments and step counts into the flat buffers the Adam launches
        read, and the optimiser state views of them again"""
        self.sa.bind(self.d.optimiser, self.d.model_actor)
        self.sc.bind(self.d.critic_optimiser, self.d.model_critic)

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)

    def sliced(self, batch):
        """whether the fp32 steps of a `batch`-row minibatch take the sliced
        schedule (sk_update_scratch_f32 > 0; what sk_actor_grad_f32_step's
        shared launch needs)"""
        return bool(self.f32) and int(self.L.sk_update_scratch_f32(int(batch), None)) > 0

    def _partial(self, batch, n_params):
        key = (batch, n_params)
        t = self._partials.get(key)
        if t is None:
            g = int(self.L.sk_update_partials_f32(batch) if self.f32 else self.L.sk_update_partials(batch))
            main = torch.empty((g, n_params), dtype=torch.float32, device=self.dev)
            scratch, rows = None, 0
            if self.f32:
                r = ctypes.c_int64(0)
                n = int(self.L.sk_update_scratch_f32(batch, ctypes.byref(r)))
                if n > 0:
                    scratch, rows = torch.empty(n, dtype=torch.float32, device=self.dev), r.value
            t = self._partials[key] = _Partials(main, scratch, rows)
        return t

    def _pack_flat(self, jobs):
        """one launch packing [(flat params, ld2, n_out, out buffer)]"""
        k = len(jobs)
        flats = (ctypes.c_void_p * k)(*[f.data_ptr() for f, _, _, _ in jobs])
        ld2s = (ctypes.c_int32 * k)(*[l for _, l, _, _ in jobs])
        nouts = (ctypes.c_int32 * k)(*[n for _, _, n, _ in jobs])
        outs = (ctypes.c_void_p * k)(*[o.data_ptr() for _, _, _, o in jobs])
        _capi.check(self.L.sk_grad_pack_flat(flats, ld2s, nouts, outs, k, self._stream()))

    @torch.no_grad()
    def pack(self):
        """full packs of every net from its parameters (at start, and after
        parameters change outside the Adam launches, e.g. load_state_dict);
        between steps each Adam launch rewrites the entries it produces"""
        if self.f32:
            return
        jobs = [(self.fa, 256, 2, self.gpa), (self.fc, 258, 1, self.gpc)]
        if self.ta is not None:
            jobs += [(self.ta, 256, 2, self.gpta), (self.tc, 258, 1, self.gptc)]
        self._pack_flat(jobs)

    def _loss_slot(self, k):
        if self._loss_private is not None:  # a captured graph's own slots (private_loss_slots)
            buf, idx = self._loss_private
            i = idx[k]
            idx[k] = (i + 1) % buf.shape[1]
            return buf[k, i]
        i = self._li[k]
        self._li[k] = (i + 1) % self.LOSS_HIST
        return self.loss_hist[k, i]

    @contextlib.contextmanager
    def private_loss_slots(self, n):
        """Steps recorded inside this context write their losses into a
        buffer of their own ([2][n], yielded; the caller keeps it with the
        graph), not into loss_hist: a captured graph rewrites its slots on
        every replay, which must not overwrite a loss an eager step returned
        (the LOSS_HIST promise)."""
        buf = torch.zeros(2, n, dtype=torch.float32, device=self.dev)
        self._loss_private = (buf, [0, 0])
        try:
            yield buf
        finally:
            self._loss_private = None

    def _packs(self, critic):
        """the packs the Adam launch of a step keeps current"""
        if self.f32:
            if critic or self.split_pack is None:
                return None
            return PackTargets(None, None, None, 256, 2, self.split_pack.data_ptr())
        if critic:
            return PackTargets(self.gpc.data_ptr(), self.gptc.data_ptr() if self.tc is not None else None, None,
                               258, 1)
        return PackTargets(self.gpa.data_ptr(), self.gpta.data_ptr() if self.ta is not None else None,
                           self.fwd_pack.data_ptr() if self.fwd_pack is not None else None, 256, 2)

    def _adam(self, part, flat, st, target, stat=None, scale=1.0, out=None, counter=None, packs=None):
        P = flat.numel()
        if not self.soft_update_in_adam:
            target = None
            if packs is not None:
                packs = PackTargets(packs.param_gpack, None, packs.actor_fwd_pack, packs.ld2, packs.n_out,
                                    packs.actor_split_pack)
        pk = ctypes.byref(packs) if packs is not None else None
        tau = float(self.d.tau) if target is not None else 0.0
        if self.d.multi():  # sum partials -> flat grad -> RCCL sum (losses are global-batch normalised) -> apply
            if self.grad_flat is None or self.grad_flat.numel() < P:
                self.grad_flat = torch.empty(max(36609, P), dtype=torch.float32, device=self.dev)
            g = self.grad_flat[:P]
            self._sum_partials(part, P, g)
            self.d.allreduce_sum(g)
            _capi.check(self.L.sk_adam_flat_packed(None, 0, P, _p(g), None, 1, _p(flat), _p(st.m), _p(st.v),
                                                   _p(st.steps), st.lr, st.b1, st.b2, st.eps, _p(target), tau,
                                                   _p(stat), float(scale), _p(out), _p(counter), pk, self._stream()))
        else:
            _capi.check(self.L.sk_adam_flat_sliced(_p(part.main), part.rows, _p(part.scratch), part.w1_rows, P, None,
                                                   None, 1, _p(flat), _p(st.m), _p(st.v), _p(st.steps), st.lr, st.b1,
                                                   st.b2, st.eps, _p(target), tau, _p(stat), float(scale), _p(out),
                                                   _p(counter), pk, self._stream()))

    def _sum_partials(self, part, P, g):
        """the flat gradient (no step) from a step's partials"""
        _capi.check(self.L.sk_adam_flat_sliced(_p(part.main), part.rows, _p(part.scratch), part.w1_rows, P, None,
                                               _p(g), 0, None, None, None, None, 0.0, 0.0, 0.0, 0.0, None, 0.0, None,
                                               0.0, None, None, None, self._stream()))

    @torch.no_grad()
    def critic_step(self, s, a, target=None, mask_out=None, s2=None, r=None, d=None, gamma=0.0, row_offset=0,
                    global_batch=None, step_job=None):
        """One critic Adam step on MSE(Q(s, a), y), Dropout active; y = target,
        or, given s2 / r / d, the bootstrap y = r + gamma (1 - d) Q'(s2,
        mu'(s2)) computed inside the same launch from the target nets.  The
        rows are global batch rows row_offset .. (their Dropout keys) of a
        global batch of global_batch rows (the loss normaliser; default this
        batch).  step_job (fp32): a prepared acting launch run in the
        gradient's backward launch (sk_critic_grad_f32_step).  Returns the
        loss (device scalar; this rank's share)."""
        s, a = s.float().contiguous(), a.float().contiguous()
        B = s.shape[0]
        gb = B if global_batch is None else int(global_batch)
        part = self._partial(B, self.fc.numel())
        st = self.sc
        if step_job is not None and not self.f32:
            raise ValueError("step_job needs the fp32 kernels")
        rc = self._critic_grad(s, a, target, s2, r, d, gamma, row_offset, gb, part, st.steps, mask_out,
                               step_job=step_job)
        _capi.check(rc)
        loss = self._loss_slot(0)
        self._adam(part, self.fc, st, self.tc, stat=self.stats[0:1], scale=1.0 / gb, out=loss, counter=self.calls,
                   packs=self._packs(critic=True))
        return loss

    # ------------------------------------------------------------ models_fit, resident
    FIT_ROWS = 16              # the resident kernels' minibatch (SkillshotLearner.py:434 batch_size=16)
    FIT_STEPS_PER_LAUNCH = 4096  # minibatch steps per resident launch (~20 ms; a progress-sized unit)

    def _fit_buffers(self):
        if getattr(self, "fit_x", None) is None:
            nb = int(self.L.sk_fit_xbuf_bytes())
            self.fit_x = torch.zeros(nb // 8, dtype=torch.int64, device=self.dev)  # granule slots, zeroed once
            self.fit_epoch = torch.zeros(1, dtype=torch.int64, device=self.dev)     # their epoch, across launches
            # [0] a lost exchange, [1] the last launch's placement (2: one XCD, 1: spread)
            self.fit_timeout = torch.zeros(2, dtype=torch.int32, device=self.dev)

    @torch.no_grad()
    def fit_critic(self, s, a, y, losses=None):
        """models_fit's critic pass (SkillshotLearner.py:419-434) over the
        full 16-row minibatches of the rows (s, a, y) in the order given:
        each minibatch one Adam step on MSE(Q(s, a), y) with Dropout active,
        in resident launches of up to FIT_STEPS_PER_LAUNCH steps
        (sk_fit_critic_f32, csrc/sk_fit.hip: the net and its moments held
        on chip by 16 workgroups).  Equal up to fp32 summation order to one
        critic_step per minibatch (no soft update: models_fit has no target
        nets).  Returns the number of minibatch steps taken; rows past the
        last full minibatch are the caller's.  losses: float [steps] (each
        step's loss) or None.  Call fit_check() before trusting the net."""
        if not self.f32:
            raise ValueError("the resident fit runs the fp32 kernels")
        b = self.FIT_ROWS
        n = int(s.shape[0]) // b
        if n == 0:
            return 0
        s, a, y = s.float().contiguous(), a.float().contiguous(), y.float().contiguous()
        self._fit_buffers()
        st = self.sc
        for k0 in range(0, n, self.FIT_STEPS_PER_LAUNCH):
            m = min(self.FIT_STEPS_PER_LAUNCH, n - k0)
            r0 = k0 * b
            _capi.check(self.L.sk_fit_critic_f32(
                _p(self.fc), _p(st.m), _p(st.v), _p(st.steps), st.steps.numel(), _p(s[r0:]), _p(a[r0:]), _p(y[r0:]),
                m, self.seed, _p(self.calls), st.lr, st.b1, st.b2, st.eps, _p(self.fit_x), _p(self.fit_epoch),
                _p(self.fit_timeout), _p(losses[k0:]) if losses is not None else None, self._stream()))
        return n

    @torch.no_grad()
    def fit_actor(self, s):
        """models_fit's actor pass (SkillshotLearner.py:386-417, 436-443) over
        the full 16-row minibatches of s: each one Adam step of the actor on
        -sum Q(s, mu(s)) with the critic as it stands (inference), in
        resident launches (sk_fit_actor_f32); then the actor's split pack is
        rewritten once (the three-launch steps rewrite it in every Adam
        launch).  Returns the number of minibatch steps taken."""
        if not self.f32:
            raise ValueError("the resident fit runs the fp32 kernels")
        b = self.FIT_ROWS
        n = int(s.shape[0]) // b
        if n == 0:
            return 0
        s = s.float().contiguous()
        self._fit_buffers()
        st = self.sa
        per = min(self.FIT_STEPS_PER_LAUNCH, n)
        z = getattr(self, "fit_z", None)
        if z is None or z.numel() < per * b * 128:  # the frozen critic's pre-activations, one launch's rows
            z = self.fit_z = torch.empty(per * b * 128, dtype=torch.float32, device=self.dev)
        for k0 in range(0, n, self.FIT_STEPS_PER_LAUNCH):
            m = min(self.FIT_STEPS_PER_LAUNCH, n - k0)
            _capi.check(self.L.sk_fit_actor_f32(
                _p(self.fa), _p(st.m), _p(st.v), _p(st.steps), st.steps.numel(), _p(self.fc), _p(s[k0 * b:]), m,
                st.lr, st.b1, st.b2, st.eps, _p(self.fit_x), _p(self.fit_epoch), _p(self.fit_timeout), _p(z),
                self._stream()))
        if self.split_pack is not None:
            _capi.check(self.L.sk_actor_split_pack_f32(_p(self.fa), _p(self.split_pack), self._stream()))
        return n

    def fit_check(self):
        """raise if a resident fit launch lost an in-launch exchange (host
        sync).  The flag is cleared as it is reported, so the next pass starts
        clean; the net that pass wrote is undefined."""
        t = getattr(self, "fit_timeout", None)
        if t is not None and int(t[0].item()):
            t[0].zero_()
            raise SkillshotError("resident models_fit: an in-launch exchange timed out; the nets are undefined")

    def fit_snapshot(self, critic):
        """a copy of what one resident pass rewrites (the net, its Adam
        moments and step counts; the critic's Dropout call number), so a pass
        that fails can be restored and rerun on the three-launch steps"""
        st = self.sc if critic else self.sa
        f = self.fc if critic else self.fa
        return (critic, f.clone(), st.m.clone(), st.v.clone(), st.steps.clone(), self.calls.clone())

    def fit_restore(self, snap):
        critic, f, m, v, steps, calls = snap
        st = self.sc if critic else self.sa
        (self.fc if critic else self.fa).copy_(f)
        st.m.copy_(m)
        st.v.copy_(v)
        st.steps.copy_(steps)
        self.calls.copy_(calls)

    @torch.no_grad()
    def critic_step_sampled(self, ring, batch, gamma=0.0, row_offset=0, global_batch=None, total=None, exclude=0,
                            step_job=None):
        """critic_step on a minibatch the launch draws from the replay ring:
        equal to ring.sample_dev(batch) followed by critic_step with the
        bootstrap target (gamma > 0) or y = r.  total: the device count the
        draw is keyed on (default the ring's); exclude > 0 leaves out the
        rows an insert running beside the step writes (sk_ring_sample).
        step_job (fp32): a prepared acting launch run in the gradient's
        backward launch (sk_critic_grad_f32_sampled_step), before the Adam
        launch.  Returns (loss, (s, a, r, s2, d)), the sample buffers."""
        B = int(batch)
        gb = B if global_batch is None else int(global_batch)
        if not 0 <= int(exclude) < ring.cap:
            raise ValueError(f"exclude {exclude} outside [0, capacity {ring.cap})")
        out, draw = ring.next_draw(B)
        tp = (total if total is not None else ring.total_t).data_ptr()
        q = RingSample(ring.buf.data_ptr(), ring.cap, tp, ring.seed, draw, *[t.data_ptr() for t in out],
                       int(exclude))
        part = self._partial(B, self.fc.numel())
        st = self.sc
        boot = gamma > 0.0
        if step_job is not None and not self.f32:
            raise ValueError("step_job needs the fp32 kernels")
        if self.f32:
            ta = (self.ta if self.ta is not None else self.fa) if boot else None
            tc = (self.tc if self.tc is not None else self.fc) if boot else None
            args = (_p(self.fc), ctypes.byref(q), float(gamma), _p(ta), _p(tc), B, int(row_offset), 2.0 / gb,
                    self.seed, _p(self.calls), _p(part.main), _p(st.steps), st.steps.numel(), _p(self.stats[0:1]),
                    None, _p(part.scratch))
            if step_job is not None:
                _capi.check(self.L.sk_critic_grad_f32_sampled_step(*args, ctypes.byref(step_job), self._stream()))
            else:
                _capi.check(self.L.sk_critic_grad_f32_sampled(*args, self._stream()))
        else:
            _capi.check(self.L.sk_critic_grad_bootstrap_sampled(
                _p(self.gpc), ctypes.byref(q), float(gamma), _p(self.gpta) if boot else None,
                _p(self.gptc) if boot else None, B, int(row_offset), 2.0 / gb, self.seed, _p(self.calls),
                _p(part.main), _p(st.steps), st.steps.numel(), _p(self.stats[0:1]), None, self._stream()))
        loss = self._loss_slot(0)
        self._adam(part, self.fc, st, self.tc, stat=self.stats[0:1], scale=1.0 / gb, out=loss, counter=self.calls,
                   packs=self._packs(critic=True))
        return loss, out

    def _critic_grad(self, s, a, target, s2, r, d, gamma, row_offset, gb, part, steps, mask_out, stat=True,
                     step_job=None):
        n_steps = steps.numel() if steps is not None else 0
        statp = _p(self.stats[0:1]) if stat else None
        if self.f32:
            boot = s2 is not None
            ta = (self.ta if self.ta is not None else self.fa) if boot else None
            tc = (self.tc if self.tc is not None else self.fc) if boot else None
            s2c = s2.float().contiguous() if boot else None
            rc_ = r.float().contiguous() if boot else None
            dc = d.float().contiguous() if boot else None
            y = None if boot else target.float().contiguous()
            args = (_p(self.fc), _p(s), _p(a), _p(y), _p(s2c), _p(rc_), _p(dc), float(gamma), _p(ta), _p(tc),
                    s.shape[0], int(row_offset), 2.0 / gb, self.seed, _p(self.calls), _p(part.main), _p(steps),
                    n_steps, statp, _p(mask_out), _p(part.scratch))
            if step_job is not None:
                return self.L.sk_critic_grad_f32_step(*args, ctypes.byref(step_job), self._stream())
            return self.L.sk_critic_grad_f32(*args, self._stream())
        if s2 is not None:
            s2c, rc_, dc = s2.float().contiguous(), r.float().contiguous(), d.float().contiguous()
            return self.L.sk_critic_grad_bootstrap(
                _p(self.gpc), _p(s), _p(a), None, _p(s2c), _p(rc_), _p(dc), float(gamma), _p(self.gpta),
                _p(self.gptc), s.shape[0], int(row_offset), 2.0 / gb, self.seed, _p(self.calls), _p(part.main), _p(steps),
                n_steps, statp, _p(mask_out), self._stream())
        y = target.float().contiguous()
        return self.L.sk_critic_grad(_p(self.gpc), _p(s), _p(a), _p(y), s.shape[0], int(row_offset), 2.0 / gb,
                                     self.seed, _p(self.calls), _p(part.main), _p(steps), n_steps, statp, _p(mask_out),
                                     self._stream())

    @torch.no_grad()
    def actor_step(self, s, before_adam=None, step_job=None):
        """One actor Adam step on -sum_b Q(s_b, mu(s_b)) (critic at inference);
        returns that loss (device scalar).  before_adam() runs between the
        gradient and the Adam launch (the overlapped tick joins the acting
        stream there: the Adam launch rewrites the weights the actor reads).
        step_job (fp32): a prepared acting launch (VecSkillshotGame.act_step
        (job=...)) run in the gradient's backward launch
        (sk_actor_grad_f32_step), before the Adam launch."""
        s = s.float().contiguous()
        B = s.shape[0]
        part = self._partial(B, self.fa.numel())
        st = self.sa
        if step_job is not None:
            if not self.f32:
                raise ValueError("step_job needs the fp32 kernels")
            rc = self.L.sk_actor_grad_f32_step(_p(self.fa), _p(self.fc), _p(s), B, 1.0, _p(part.main), _p(st.steps),
                                               st.steps.numel(), _p(self.stats[1:]), _p(part.scratch),
                                               ctypes.byref(step_job), self._stream())
        else:
            rc = self._actor_grad(s, part, st.steps, self.stats[1:])
        _capi.check(rc)
        if before_adam is not None:
            before_adam()
        loss = self._loss_slot(1)
        self._adam(part, self.fa, st, self.ta, stat=self.stats[1:], scale=-1.0, out=loss,
                   packs=self._packs(critic=False))
        return loss

    def _actor_grad(self, s, part, steps, stat):
        n = steps.numel() if steps is not None else 0
        if self.f32:
            return self.L.sk_actor_grad_f32(_p(self.fa), _p(self.fc), _p(s), s.shape[0], 1.0, _p(part.main), _p(steps),
                                            n, _p(stat), _p(part.scratch), self._stream())
        return self.L.sk_actor_grad(_p(self.gpa), _p(self.gpc), _p(s), s.shape[0], 1.0, _p(part.main), _p(steps), n,
                                    _p(stat), self._stream())

    @torch.no_grad()
    def grads(self, which, s, a=None, target=None, mask_out=None, s2=None, r=None, d=None, gamma=0.0, row_offset=0,
              global_batch=None):
        """Test hook: the flat gradient the kernels compute, without stepping
        (the Adam step counters are not touched; the critic's Dropout call
        number advances as a step would)."""
        B = s.shape[0]
        if which == "critic":
            flat = self.fc
            part = self._partial(B, flat.numel())
            gb = B if global_batch is None else int(global_batch)
            rc = self._critic_grad(s.float().contiguous(), a.float().contiguous(), target, s2, r, d, gamma,
                                   row_offset, gb, part, None, mask_out, stat=False)
            _capi.check(rc)
            self.calls.add_(1)
        else:
            flat = self.fa
            part = self._partial(B, flat.numel())
            _capi.check(self._actor_grad(s.float().contiguous(), part, None, None))
        g = torch.empty_like(flat)
        self._sum_partials(part, flat.numel(), g)
        return g
