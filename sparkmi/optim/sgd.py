"""SGD over a :class:`FlatParams` buffer (torch.optim.SGD semantics; the reference uses plain
SGD without momentum: distributed_multilayer_perceptron.py:111, distributed_cnn.py:138)."""
import torch

from .. import _native
from .adam import _FlatOptimizer


class SGD(_FlatOptimizer):
    def __init__(self, flat, lr=0.01, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False):
        super().__init__(flat, lr)
        self.momentum, self.dampening, self.weight_decay, self.nesterov = momentum, dampening, weight_decay, nesterov
        self.buf = torch.zeros_like(flat.master) if momentum else None

    def step(self):
        f = self.flat
        if _native.use_native(f.master):
            C = _native.C()
            st = _native.stream()
            C.sgd(f.master.data_ptr(), f.grad.data_ptr(), _native.ptr(self.buf), _native.ptr(f.shadow), f.numel,
                  self.lr_t.data_ptr(), self.step_t.data_ptr(), self.done_t.data_ptr(), self.momentum, self.dampening, self.weight_decay,
                  int(self.nesterov), self.grad_scale, int(self.zero_grad_after_step), _native.ptr(f.planes),
                  f.plane_stride(), _native.ptr(self.bump_seed), st)
            return
        with torch.no_grad():
            self.step_t.add_(1)
            if self.bump_seed is not None:
                self.bump_seed.add_(1)
            lr = float(self.lr_t.item())
            d = f.grad * self.grad_scale
            if self.weight_decay:
                d = d + self.weight_decay * f.master
            if self.momentum:
                if float(self.step_t.item()) <= 1:
                    self.buf.copy_(d)
                else:
                    self.buf.mul_(self.momentum).add_(d, alpha=1 - self.dampening)
                d = d + self.momentum * self.buf if self.nesterov else self.buf
            f.master.add_(d, alpha=-lr)
            if self.zero_grad_after_step:
                f.grad.zero_()
            if f.shadow is not None:
                f.shadow.copy_(f.master.to(torch.bfloat16))
            f.refresh_planes()

    def state_dict(self):
        sd = super().state_dict()
        if self.buf is not None:
            sd["momentum_buffer"] = self.buf.clone()
        return sd

    def load_state_dict(self, sd):
        super().load_state_dict(sd)
        if self.buf is not None and "momentum_buffer" in sd:
            self.buf.copy_(sd["momentum_buffer"])
