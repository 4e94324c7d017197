"""Multilayer perceptron classifier (the reference's ``Multilayer_perceptor``:
distributed_multilayer_perceptron.py:44-53 — Linear(4,5) -> Sigmoid -> Linear(5,4) -> Sigmoid
-> Linear(4,3), logits out).  Same attribute names (layer_1.., sigmoid) so reference
state_dicts load.  ``forward`` returns logits; ``loss`` runs the fused HIP MLP+CE kernels.
"""
import torch
from torch import nn

from ..ops.mlp import mlp_grad_step, mlp_logits, mlp_loss, mlp_sgd_step


# steps per launch of the multi-step SGD kernel (csrc/include/smi_mlp.h MLP_MAX_STEPS)
MLP_MAX_STEPS = 32

class MultilayerPerceptron(nn.Module):
    def __init__(self, layers=(4, 5, 4, 3), activation="sigmoid"):
        super().__init__()
        self.layer_sizes = list(layers)
        self.activation = activation
        for i in range(len(layers) - 1):
            setattr(self, f"layer_{i + 1}", nn.Linear(layers[i], layers[i + 1]))
        self.sigmoid = nn.Sigmoid()

    def linears(self):
        return [getattr(self, f"layer_{i + 1}") for i in range(len(self.layer_sizes) - 1)]

    def forward(self, x):
        lins = self.linears()
        if x.is_cuda:
            return mlp_logits(x, [l.weight for l in lins], [l.bias for l in lins], self.activation)
        h = x
        for i, l in enumerate(lins):
            h = l(h)
            if i < len(lins) - 1:
                h = torch.sigmoid(h) if self.activation == "sigmoid" else torch.relu(h)
        return h

    def loss(self, x, y, row_weight=None):
        lins = self.linears()
        return mlp_loss(x, y, [l.weight for l in lins], [l.bias for l in lins], self.activation, row_weight)


    def _fused_sgd_ok(self, opt, x):
        from .. import _native
        from ..optim.sgd import SGD
        flat = getattr(opt, "flat", None)
        return (x.is_cuda and isinstance(opt, SGD) and not opt.momentum and not opt.weight_decay
                and getattr(opt, "ranges", None) is None and (flat is None or flat.shadow is None)
                and _native.use_native(x))

    def gather_in_step(self, opt, ddp, x):
        """True when every training step will run as the multi-step SGD kernel reading its shuffled
        rows from the dataset itself (index mode: perm[cursor * B + i]; sparkmi/train/trainer.py
        with a DeviceLoader(fixed=True)): single executor, plain SGD, the 4-5-4-3 shape, B <= 64."""
        dims = [self.linears()[0].weight.shape[1]] + [l.weight.shape[0] for l in self.linears()]
        return (ddp is None and x.dim() == 2 and x.dtype == torch.float32 and x.shape[0] <= 64
                and dims == [4, 5, 4, 3] and self._fused_sgd_ok(opt, x))

    def fused_sgd_step(self, opt, x, y):
        """The whole training step — forward, CE, backward, SGD update — as ONE HIP launch
        (csrc/kernels/mlp.hip mode 2); the loss of the step is returned.  None when it does not
        apply (CPU, an optimizer other than plain SGD, a bf16 shadow to refresh): the caller
        then runs the usual forward/backward/step."""
        if getattr(x, "_smi_gather", None) is not None:  # index mode: a one-step multi-step launch
            return self.fused_sgd_steps(opt, [(x, y)])[0]
        if not self._fused_sgd_ok(opt, x):
            return None
        lins = self.linears()
        return mlp_sgd_step(x, y, [l.weight for l in lins], [l.bias for l in lins], opt.lr_t, opt.step_t,
                            self.activation, grad_scale=opt.grad_scale)


    def fused_sgd_steps(self, opt, batches):
        """Several consecutive fused SGD steps (one per (x, y) of ``batches``) as ONE launch
        (csrc/kernels/mlp.hip mlp_small_steps_kernel): bitwise the steps of ``fused_sgd_step`` one
        after another.  Returns the per-step losses, or None when it does not apply (the caller
        then runs the steps one by one)."""
        from ..ops.mlp import mlp_sgd_steps
        lins = self.linears()
        g = getattr(batches[0][0], "_smi_gather", None)
        if g is not None:
            # index mode: every batch is the fixed loader's (empty) buffer; the kernel reads the rows
            if any(getattr(b[0], "_smi_gather", None) is not g for b in batches):
                raise RuntimeError("MultilayerPerceptron: index-mode and ordinary batches mixed")
            # the kernel runs at most MLP_MAX_STEPS steps per launch: a longer group (Trainer unroll
            # > 32) is several consecutive launches, each advancing the device cursor
            from ..ops.mlp import StepLosses
            out, totals = StepLosses(), []
            for i0 in range(0, len(batches), MLP_MAX_STEPS):
                part = mlp_sgd_steps([(g[1], g[2])], [l.weight for l in lins], [l.bias for l in lins], opt.lr_t,
                                     opt.step_t, self.activation, grad_scale=opt.grad_scale,
                                     index=(g[0], g[3], g[4], min(MLP_MAX_STEPS, len(batches) - i0)))
                if part is None:
                    raise RuntimeError("MultilayerPerceptron: index-mode batch but the fused step does not apply")
                out.extend(part)
                totals.append(part.total)
            out.total = totals[0] if len(totals) == 1 else torch.stack([t.reshape(()) for t in totals]).sum()
            return out
        if (len(batches) > MLP_MAX_STEPS or not all(self._fused_sgd_ok(opt, b[0]) for b in batches)
                or len({b[0].data_ptr() for b in batches}) != len(batches)):
            return None
        return mlp_sgd_steps(batches, [l.weight for l in lins], [l.bias for l in lins], opt.lr_t, opt.step_t,
                             self.activation, grad_scale=opt.grad_scale)

    def fused_grad_step(self, x, y):
        """Forward, CE and backward as ONE HIP launch, the gradients added to the flat gradient
        buffer (the data-parallel step's local half: the IPC all-reduce and SGD follow).  None when
        it does not apply (CPU, parameters outside a FlatParams buffer)."""
        from .. import _native
        if not x.is_cuda or not _native.use_native(x) or getattr(self, "_smi_flat", None) is None:
            return None
        lins = self.linears()
        return mlp_grad_step(x, y, [l.weight for l in lins], [l.bias for l in lins], self.activation)


Multilayer_perceptor = MultilayerPerceptron  # reference class name
