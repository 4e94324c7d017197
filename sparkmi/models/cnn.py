"""FashionMNISTModel — the reference CNN (distributed_cnn.py:47-86, pytorch_cnn.py:12-49) with the
same module names (block_1 / block_2 / classifier, nn.Sequential indices) so reference
state_dicts load.  ``loss(x, y)`` runs the fused whole-network HIP kernel (sparkmi/ops/cnn.py);
``forward(x)`` returns logits (fused inference kernel on GPU, torch ops on CPU).
``dtype="bf16"`` (the BASELINE CNN config) runs the four convolutions on bf16 matrix cores
(implicit GEMM on v_mfma_f32_16x16x32_bf16, fp32 accumulation) inside the same fused kernel.
"""
import torch
from torch import nn

from ..ops.cnn import cnn_grad_step, cnn_logits, cnn_loss, cnn_sgd_step


class FashionMNISTModel(nn.Module):
    def __init__(self, input_shape: int = 1, hidden_units: int = 10, output_shape: int = 10, dtype: str = "fp32"):
        super().__init__()
        if dtype not in ("fp32", "bf16"):
            raise ValueError(f"dtype must be 'fp32' or 'bf16', got {dtype!r}")
        self.conv_dtype = dtype  # GPU: "bf16" runs the convolutions on bf16 matrix cores
        self.block_1 = nn.Sequential(
            nn.Conv2d(input_shape, hidden_units, kernel_size=3, stride=1, padding=1), nn.ReLU(),
            nn.Conv2d(hidden_units, hidden_units, kernel_size=3, stride=1, padding=1), nn.ReLU(),
            nn.MaxPool2d(kernel_size=2, stride=2))
        self.block_2 = nn.Sequential(
            nn.Conv2d(hidden_units, hidden_units, 3, padding=1), nn.ReLU(),
            nn.Conv2d(hidden_units, hidden_units, 3, padding=1), nn.ReLU(),
            nn.MaxPool2d(2))
        self.classifier = nn.Sequential(nn.Flatten(), nn.Linear(hidden_units * 7 * 7, output_shape))
        # the fused step's counters (re-armed by the kernel): CNN_TICKS for the tail, then 3 per
        # image (batch <= CNN_MAXB = 64; csrc/include/smi_cnn.h); per model, so two models never
        # share them; not part of the state_dict (reference key parity)
        # for the weight-gradient helpers' hand-off flags
        self.register_buffer("_step_tick", torch.zeros(34 + 3 * 64, dtype=torch.int32), persistent=False)

    def param_list(self):
        c = [self.block_1[0], self.block_1[2], self.block_2[0], self.block_2[2], self.classifier[1]]
        out = []
        for m in c:
            out += [m.weight, m.bias]
        return out

    def forward(self, x):
        return cnn_logits(x, self.param_list(), self.conv_dtype == "bf16")

    def fused_batch_limit(self):
        """The largest batch the one-launch fused step takes for this model and its dtype (the
        fused tail stages every image's fc row in the kernel's LDS; csrc/kernels/cnn.hip
        smi_cnn_max_batch); 0 without the native library."""
        from .. import _native
        if not _native.has_native():
            return 0
        p = self.param_list()
        return int(_native.C().cnn_max_batch(p[0].shape[0], p[0].shape[1], p[8].shape[0], int(self.conv_dtype == "bf16")))

    def _fused_ok(self, bs):
        """Whether a fused step takes batch ``bs``; warns once per model when the batch alone (past
        fused_batch_limit) sends an otherwise fused-eligible step to the multi-launch path."""
        from .. import _native
        p = self.param_list()
        ok = bool(_native.C().cnn_fused_ok(p[0].shape[0], p[0].shape[1], p[8].shape[0], bs,
                                           int(self.conv_dtype == "bf16")))
        if not ok and not getattr(self, "_warned_batch", False):
            lim = self.fused_batch_limit()
            if lim and bs > lim:
                import warnings
                warnings.warn(f"FashionMNISTModel: batch {bs} exceeds the fused step's limit {lim} for this model "
                              f"({self.conv_dtype}); running the multi-launch step", RuntimeWarning, stacklevel=3)
                self._warned_batch = True
        return ok

    def gather_in_step(self, opt, ddp, x):
        """True when every training step of this model will run as one of its fused kernels, which
        then read their shuffled batch straight from the dataset (index mode: perm[cursor * B + i],
        device cursor advanced by the kernel) — the loop needs no separate gather launch
        (sparkmi/train/trainer.py with a DeviceLoader(fixed=True))."""
        from .. import _native
        from ..optim.sgd import SGD
        params = self.param_list()
        if (not x.is_cuda or not _native.use_native(x) or x.dim() != 4 or getattr(self, "_smi_flat", None) is None
                or not self._fused_ok(x.shape[0])):
            return False
        if ddp is not None:
            return True  # fused_grad_step
        flat = opt.flat
        return (isinstance(opt, SGD) and not opt.momentum and not opt.weight_decay and opt.grad_scale == 1.0
                and getattr(opt, "ranges", None) is None and getattr(flat, "planes", None) is None)

    @staticmethod
    def _gather(x, y):
        """(x, y, index) for the fused kernels: the dataset and (batch, perm, cursor) when ``x`` is a
        fixed loader's batch buffer in index mode, else the batch itself."""
        g = getattr(x, "_smi_gather", None)
        if g is None:
            return x, y, None
        return g[1], g[2], (g[0], g[3], g[4])

    def fused_sgd_step(self, opt, x, y):
        """The whole single-executor training step (forward, CE, backward, batch gradient sum,
        SGD update) as ONE HIP launch (csrc/kernels/cnn.hip, fused tail); returns the loss.  None
        when it does not apply (CPU, data parallelism, an optimizer other than plain SGD, a batch
        whose fc activations do not fit the kernel's LDS): the caller runs the usual forward / backward / step."""
        from .. import _native
        from ..optim.sgd import SGD
        flat = getattr(opt, "flat", None)
        params = self.param_list()
        x, y, index = self._gather(x, y)
        bs = index[0] if index is not None else x.shape[0]
        if (not x.is_cuda or not _native.use_native(x) or not isinstance(opt, SGD) or opt.momentum
                or opt.weight_decay or opt.grad_scale != 1.0 or getattr(opt, "ranges", None) is not None
                or flat is None or getattr(flat, "planes", None) is not None or x.dim() != 4
                or not self._fused_ok(bs)):
            if index is not None:
                raise RuntimeError("FashionMNISTModel: index-mode batch but the fused step does not apply")
            return None
        shadows = None
        if flat.shadow is not None:
            offs = [flat.offsets[flat.index[id(p)]] for p in params]
            shadows = [flat.shadow[o:o + p.numel()] for p, o in zip(params, offs)]
        return cnn_sgd_step(x.contiguous(), y.to(torch.int64).contiguous(), params, opt.lr_t, opt.step_t,
                            self._step_tick, shadows, self.conv_dtype == "bf16", index)

    def fused_grad_step(self, x, y):
        """Forward, mean CE, backward and the batch gradient sum as ONE HIP launch, the gradient
        added to the parameters' flat fp32 gradient slices (the data-parallel step's local half:
        all-reduce and optimizer follow; csrc/kernels/cnn.hip gradient mode).  Returns the loss,
        or None when it does not apply (CPU, parameters outside a FlatParams buffer, a batch the
        kernel's LDS cannot stage): the caller then runs loss() and backward()."""
        from .. import _native
        from ..ops._grad import grad_buf
        params = self.param_list()
        x, y, index = self._gather(x, y)
        bs = index[0] if index is not None else x.shape[0]
        if (not x.is_cuda or not _native.use_native(x) or x.dim() != 4
                or getattr(self, "_smi_flat", None) is None
                or not self._fused_ok(bs)):
            if index is not None:
                raise RuntimeError("FashionMNISTModel: index-mode batch but the fused step does not apply")
            return None
        grads = [grad_buf(p) for p in params]
        return cnn_grad_step(x.contiguous(), y.to(torch.int64).contiguous(), params, grads, self._step_tick,
                             self.conv_dtype == "bf16", index)

    def loss(self, x, y):
        """Mean CE over the batch (distributed_cnn.py:141,177)."""
        return cnn_loss(x, y, self.param_list(), self.conv_dtype == "bf16")


CNN = FashionMNISTModel
