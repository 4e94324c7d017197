"""Adam / AdamW over a :class:`FlatParams` buffer.

torch.optim.Adam semantics (pytorch_machine_translator.py:129, distributed_lstm.py:141):
m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps).
``grad_scale`` multiplies the gradient first (1/world for data-parallel averaging folded in).
lr and the step counter are device tensors, so the update is HIP-graph capturable.
"""
import torch

from .. import _native


class _FlatOptimizer:
    def __init__(self, flat, lr):
        self.flat = flat
        dev = flat.device
        self.lr_t = torch.tensor([float(lr)], dtype=torch.float32, device=dev)
        self.step_t = torch.zeros(1, dtype=torch.float32, device=dev)
        # ticket word of the update kernel's in-kernel step advance (csrc/kernels/optim.hip)
        self.done_t = torch.zeros(1, dtype=torch.int32, device=dev)
        self.grad_scale = 1.0
        self.zero_grad_after_step = True
        # the model's dropout step seed (an int32 device tensor), advanced by the update kernel for
        # the next step (set by StepRunner; None: the runner advances it with its own launch)
        self.bump_seed = None

    @property
    def lr(self):
        return float(self.lr_t.item())

    def set_lr(self, lr):
        self.lr_t.fill_(float(lr))

    def zero_grad(self, set_to_none=False):
        self.flat.zero_grad()

    def state_dict(self):
        return {"lr": self.lr_t.clone(), "step": self.step_t.clone()}

    def load_state_dict(self, sd):
        self.lr_t.copy_(sd["lr"])
        self.step_t.copy_(sd["step"])


class Adam(_FlatOptimizer):
    adamw = False

    def __init__(self, flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(flat, lr)
        self.b1, self.b2 = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.m = torch.zeros_like(flat.master)
        self.v = torch.zeros_like(flat.master)
        self.ranges = None
        self._early = []  # flat ranges already updated this step (step_ranges); step() does the rest

    def shard(self, ranges):
        """ZeRO-1: update only the [start, end) ranges of the flat buffer (this data-parallel
        rank's pieces, sparkmi/parallel/ddp.py); the moments are kept for those ranges only, in
        one compact buffer, and the update is ONE multi-range launch with one step advance."""
        self.ranges = [(int(s), int(e)) for s, e in ranges]
        offs, o = [], 0
        for s, e in self.ranges:
            offs.append(o)
            o += e - s
        self._moff = offs
        self.m = torch.zeros(o, dtype=torch.float32, device=self.flat.device)
        self.v = torch.zeros(o, dtype=torch.float32, device=self.flat.device)
        return self

    def _multi(self, ranges, moff, advance):
        """Update the flat ranges [s, e) (moments at moff) in launches of <= 64 ranges; only the
        last launch advances the step counter (and the dropout seed) when ``advance``."""
        f = self.flat
        C = _native.C()
        mp, gp, sp = f.master.data_ptr(), f.grad.data_ptr(), _native.ptr(f.shadow)
        for i in range(0, len(ranges), 64):
            rs, os_ = ranges[i:i + 64], moff[i:i + 64]
            last = advance and i + 64 >= len(ranges)
            C.adam_multi([mp + 4 * s for s, _ in rs], [gp + 4 * s for s, _ in rs],
                         [self.m.data_ptr() + 4 * o for o in os_], [self.v.data_ptr() + 4 * o for o in os_],
                         [sp + 2 * s if sp else 0 for s, _ in rs], [e - s for s, e in rs],
                         self.lr_t.data_ptr(), self.step_t.data_ptr(), self.done_t.data_ptr(), self.b1, self.b2,
                         self.eps, self.weight_decay, self.grad_scale, int(self.adamw), int(self.zero_grad_after_step),
                         [_native.ptr(f.planes) + 2 * s for s, _ in rs] if f.planes is not None else [],
                         f.plane_stride(), _native.ptr(self.bump_seed) if last else 0, int(last), _native.stream())

    def _torch_ranges(self, ranges, moff, t):
        """CPU / fallback update of flat ranges at step count t (no advance)."""
        f = self.flat
        with torch.no_grad():
            lr = float(self.lr_t.item())
            bc1, bc2 = 1 - self.b1 ** t, 1 - self.b2 ** t
            for (s, e), o in zip(ranges, moff):
                p, g = f.master[s:e], f.grad[s:e] * self.grad_scale
                m, v = self.m[o:o + e - s], self.v[o:o + e - s]
                if self.weight_decay:
                    if self.adamw:
                        p.mul_(1 - lr * self.weight_decay)
                    else:
                        g = g + self.weight_decay * p
                m.mul_(self.b1).add_(g, alpha=1 - self.b1)
                v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
                p.addcdiv_(m, v.sqrt() / (bc2 ** 0.5) + self.eps, value=-lr / bc1)
                if self.zero_grad_after_step:
                    f.grad[s:e].zero_()
                if f.shadow is not None:
                    f.shadow[s:e].copy_(p.to(torch.bfloat16))

    def _advance_torch(self):
        with torch.no_grad():
            self.step_t.add_(1)
            if self.bump_seed is not None:
                self.bump_seed.add_(1)
        return float(self.step_t.item())

    def _step_shard(self):
        f = self.flat
        if _native.use_native(f.master):
            self._multi(self.ranges, self._moff, True)
            return
        t = self._advance_torch()
        self._torch_ranges(self.ranges, self._moff, t)
        f.refresh_planes()

    def _domain(self):
        """The flat ranges this optimizer updates and their moment offsets (ZeRO-1: the owned
        pieces, compact moments; otherwise the whole buffer)."""
        if self.ranges is None:
            return [(0, self.flat.numel)], [0]
        return self.ranges, self._moff

    def _moffs(self, ranges):
        """Moment offsets of flat ranges that lie inside the update domain."""
        if self.ranges is None:
            return [s for s, _ in ranges]
        out = []
        for s, e in ranges:
            for (rs, re_), o in zip(self.ranges, self._moff):
                if rs <= s and e <= re_:
                    out.append(o + s - rs)
                    break
            else:
                raise ValueError(f"step_ranges: [{s}, {e}) is not inside an owned (ZeRO-1) piece")
        return out

    def step_ranges(self, ranges):
        """Update the parameters in the flat ranges [s, e) NOW, ahead of this step's ``step()``
        (their gradients are final while the backward, or the reduction of other gradient
        buckets, still runs): same step count and bias corrections, the counter is advanced by
        ``step()``, which then updates only the rest of the domain.  ZeRO-1: the ranges must lie
        inside owned pieces.  Element for element the same arithmetic as the one-launch update
        (tests pin it bitwise)."""
        ranges = [(int(s), int(e)) for s, e in ranges if e > s]
        if not ranges:
            return
        moff = self._moffs(ranges)
        if _native.use_native(self.flat.master):
            self._multi(ranges, moff, False)
        else:
            self._torch_ranges(ranges, moff, float(self.step_t.item()) + 1)
            self.flat.refresh_planes()
        self._early.extend(ranges)

    def _rest(self):
        """The parts of the update domain not updated by step_ranges this step (sorted, merged)
        and their moment offsets."""
        done = sorted(self._early)
        self._early = []
        out, offs = [], []
        for (ds, de), o in zip(*self._domain()):
            pos = ds
            for s, e in done:
                if e <= ds or s >= de:
                    continue
                if s > pos:
                    out.append((pos, s))
                    offs.append(o + pos - ds)
                pos = max(pos, e)
            if pos < de:
                out.append((pos, de))
                offs.append(o + pos - ds)
        return out, offs

    def step(self):
        f = self.flat
        if self._early:
            rest, roff = self._rest()
            if _native.use_native(f.master):
                if rest:
                    self._multi(rest, roff, True)
                else:  # everything went early: the counter (and the seed) still advance once
                    C = _native.C()
                    C.step_inc(self.step_t.data_ptr(), _native.stream())
                    if self.bump_seed is not None:
                        C.seed_inc(self.bump_seed.data_ptr(), _native.stream())
                return
            t = self._advance_torch()
            self._torch_ranges(rest, roff, t)
            f.refresh_planes()
            return
        if self.ranges is not None:
            return self._step_shard()
        if _native.use_native(f.master):
            C = _native.C()
            st = _native.stream()
            C.adam(f.master.data_ptr(), f.grad.data_ptr(), self.m.data_ptr(), self.v.data_ptr(), _native.ptr(f.shadow),
                   f.numel, self.lr_t.data_ptr(), self.step_t.data_ptr(), self.done_t.data_ptr(), self.b1, self.b2, self.eps,
                   self.weight_decay, self.grad_scale, int(self.adamw), int(self.zero_grad_after_step),
                   _native.ptr(f.planes), f.plane_stride(), _native.ptr(self.bump_seed), st)
            return
        with torch.no_grad():
            self.step_t.add_(1)
            if self.bump_seed is not None:
                self.bump_seed.add_(1)
            t = float(self.step_t.item())
            lr = float(self.lr_t.item())
            g = f.grad * self.grad_scale
            p = f.master
            if self.weight_decay:
                if self.adamw:
                    p.mul_(1 - lr * self.weight_decay)
                else:
                    g = g + self.weight_decay * p
            self.m.mul_(self.b1).add_(g, alpha=1 - self.b1)
            self.v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            bc1 = 1 - self.b1 ** t
            bc2 = 1 - self.b2 ** t
            denom = self.v.sqrt() / (bc2 ** 0.5) + self.eps
            p.addcdiv_(self.m, denom, value=-lr / bc1)
            if self.zero_grad_after_step:
                f.grad.zero_()
            if f.shadow is not None:
                f.shadow.copy_(p.to(torch.bfloat16))
            f.refresh_planes()

    def state_dict(self):
        sd = super().state_dict()
        sd.update(m=self.m.clone(), v=self.v.clone())
        return sd

    def load_state_dict(self, sd):
        super().load_state_dict(sd)
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])


class AdamW(Adam):
    adamw = True
