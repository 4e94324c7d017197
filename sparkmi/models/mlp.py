"""Multilayer perceptron classifier (the reference's ``Multilayer_perceptor``:
distributed_multilayer_perceptron.py:44-53 — Linear(4,5) -> Sigmoid -> Linear(5,4) -> Sigmoid
-> Linear(4,3), logits out).  Same attribute names (layer_1.., sigmoid) so reference
state_dicts load.  ``forward`` returns logits; ``loss`` runs the fused HIP MLP+CE kernels.
"""
import torch
from torch import nn

from ..ops.mlp import mlp_grad_step, mlp_logits, mlp_loss, mlp_sgd_step


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


    def fused_sgd_step(self, opt, x, y):
        """The whole training step — forward, CE, backward, SGD update — as ONE HIP launch
        (csrc/kernels/mlp.hip mode 2); the loss of the step is returned.  None when it does not
        apply (CPU, an optimizer other than plain SGD, a bf16 shadow to refresh): the caller
        then runs the usual forward/backward/step."""
        from .. import _native
        from ..optim.sgd import SGD
        flat = getattr(opt, "flat", None)
        if (not x.is_cuda or not isinstance(opt, SGD) or opt.momentum or opt.weight_decay
                or getattr(opt, "ranges", None) is not None or (flat is not None and flat.shadow is not None)
                or not _native.use_native(x)):
            return None
        lins = self.linears()
        return mlp_sgd_step(x, y, [l.weight for l in lins], [l.bias for l in lins], opt.lr_t, opt.step_t,
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
