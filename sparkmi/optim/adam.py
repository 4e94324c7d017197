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

    def _step_shard(self):
        f = self.flat
        if _native.use_native(f.master):
            C = _native.C()
            mp, gp, sp = f.master.data_ptr(), f.grad.data_ptr(), _native.ptr(f.shadow)
            C.adam_multi([mp + 4 * s for s, _ in self.ranges], [gp + 4 * s for s, _ in self.ranges],
                         [self.m.data_ptr() + 4 * o for o in self._moff], [self.v.data_ptr() + 4 * o for o in self._moff],
                         [sp + 2 * s if sp else 0 for s, _ in self.ranges], [e - s for s, e in self.ranges],
                         self.lr_t.data_ptr(), self.step_t.data_ptr(), self.done_t.data_ptr(), self.b1, self.b2,
                         self.eps, self.weight_decay, self.grad_scale, int(self.adamw), int(self.zero_grad_after_step),
                         [_native.ptr(f.planes) + 2 * s for s, _ in self.ranges] if f.planes is not None else [],
                         f.plane_stride(), _native.ptr(self.bump_seed), _native.stream())
            return
        with torch.no_grad():
            self.step_t.add_(1)
            if self.bump_seed is not None:
                self.bump_seed.add_(1)
            t = float(self.step_t.item())
            lr = float(self.lr_t.item())
            bc1, bc2 = 1 - self.b1 ** t, 1 - self.b2 ** t
            for (s, e), o in zip(self.ranges, self._moff):
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
            f.refresh_planes()

    def step(self):
        f = self.flat
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
