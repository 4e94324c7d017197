"""Softmax cross-entropy with ignore_index, mean over non-ignored targets.

Reference: CrossEntropyLoss(ignore_index=0, reduction='none') + masked mean
(pytorch_machine_translator.py:125-126,182-188) and plain mean CE
(distributed_cnn.py:141, distributed_lstm.py:142).  GPU: csrc/kernels/cross_entropy.hip —
online logsumexp forward (loss accumulated on the device, valid-row count on the device),
recompute-softmax backward writing the logit gradient in one pass.
"""
import torch

from .. import _native


class CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        V = logits.shape[-1]
        x2 = logits.reshape(-1, V)
        lab = labels.reshape(-1).to(torch.int64).contiguous()
        M = x2.shape[0]
        ctx.ignore = ignore_index
        ctx.native = _native.use_native(logits) and logits.dtype in (torch.bfloat16, torch.float32)
        if ctx.native:
            C = _native.C()
            x2 = x2.contiguous()
            lse = torch.empty(M, device=x2.device, dtype=torch.float32)
            stats = torch.empty(1, device=x2.device, dtype=torch.float32)  # valid-row count
            loss = torch.empty((), device=x2.device, dtype=torch.float32)  # its own buffer: no copy kernel
            row_loss = torch.empty(M, device=x2.device, dtype=torch.float32)
            C.ce_fwd(x2.data_ptr(), int(x2.dtype == torch.bfloat16), lab.data_ptr(), M, V, ignore_index,
                     lse.data_ptr(), stats.data_ptr(), loss.data_ptr(), row_loss.data_ptr(), _native.stream())
            ctx.save_for_backward(x2, lab, lse, stats)
            ctx.shape = logits.shape
            return loss
        xf = x2.float()
        lse = torch.logsumexp(xf, dim=-1)
        valid = lab != ignore_index
        safe = torch.where(valid, lab, torch.zeros_like(lab))
        rl = (lse - xf.gather(1, safe[:, None]).squeeze(1)) * valid.float()
        count = valid.float().sum()
        ctx.save_for_backward(x2, lab, lse, count.reshape(1))
        ctx.shape = logits.shape
        return (rl.sum() / count.clamp_min(1.0)).to(torch.float32)

    @staticmethod
    def backward(ctx, dloss):
        x2, lab, lse, stats = ctx.saved_tensors
        M, V = x2.shape
        if ctx.native:
            C = _native.C()
            grad = torch.empty_like(x2)
            dl = dloss.reshape(1).to(torch.float32).contiguous()
            # fp32: the gradient's split planes (k-padded: V is the K of the vocab projection's
            # dgrad) for the split-plane GEMMs, written by the same kernel
            from . import gemm as G
            from . import planes as _pl
            gp = _pl.new(M, V, x2.device, kpad=True) if (x2.dtype == torch.float32 and G.SP) else None
            only = gp is not None and _pl.grad_planes_ok(x2)  # dlogits feeds only the vocab dgrad / wgrad
            C.ce_bwd(x2.data_ptr(), int(x2.dtype == torch.bfloat16), lab.data_ptr(), M, V, ctx.ignore, lse.data_ptr(),
                     stats[0:1].data_ptr(), dl.data_ptr(), 0 if only else grad.data_ptr(), _native.ptr(gp),
                     gp.stride(1) if gp is not None else 0, gp.stride(0) if gp is not None else 0, _native.stream())
            if gp is not None:
                _pl.attach(grad, gp)
                grad._smi_planes_only = only
            return grad.reshape(ctx.shape), None, None
        count = stats[0].clamp_min(1.0)
        p = torch.exp(x2.float() - lse[:, None])
        valid = lab != ctx.ignore
        safe = torch.where(valid, lab, torch.zeros_like(lab))
        p[torch.arange(M), safe] -= 1.0
        p = p * (valid.float() * dloss / count)[:, None]
        return p.to(x2.dtype).reshape(ctx.shape), None, None


def cross_entropy(logits, labels, ignore_index=-100):
    return CrossEntropyFn.apply(logits, labels, int(ignore_index))
