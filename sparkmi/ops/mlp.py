"""Fused small-MLP (affine + sigmoid/relu hidden layers + affine logits + softmax-CE).

One HIP launch computes the (weighted) mean cross-entropy of a whole minibatch or full batch;
one launch recomputes the forward and accumulates every weight/bias gradient
(csrc/kernels/mlp.hip).  Used by the reference MLP (distributed_multilayer_perceptron.py:44-53)
and by the MLlib-compatible MultilayerPerceptronClassifier's L-BFGS objective.
``row_weight`` implements MLlib's per-block loss averaging.
"""
import torch

from .. import _native
from ._grad import grad_buf, grad_ready

ACT = {"sigmoid": 2, "relu": 1}


def _ref_logits(x, Ws, bs, act):
    h = x.float()
    for i, (W, b) in enumerate(zip(Ws, bs)):
        h = h @ W.float().t() + b.float()
        if i < len(Ws) - 1:
            h = torch.sigmoid(h) if act == 2 else torch.relu(h)
    return h


class MLPLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y, row_weight, act, nlayers, *params):
        Ws, bs = list(params[:nlayers]), list(params[nlayers:])
        ctx.act, ctx.nlayers = act, nlayers
        ctx.native = _native.use_native(x)
        x = x.float().contiguous()
        y = y.to(torch.int64).contiguous()
        ctx.save_for_backward(x, y, row_weight, *params)
        if ctx.native:
            loss = torch.empty(1, device=x.device, dtype=torch.float32)  # written by the kernel
            dims = [Ws[0].shape[1]] + [W.shape[0] for W in Ws]
            _native.C().mlp(0, x.data_ptr(), y.data_ptr(), _native.ptr(row_weight), x.shape[0], dims,
                            [W.data_ptr() for W in Ws], [b.data_ptr() for b in bs], [], [], 0, loss.data_ptr(), 0,
                            act, _native.stream())
            return loss[0]
        z = _ref_logits(x, Ws, bs, act)
        rl = torch.logsumexp(z, 1) - z.gather(1, y[:, None]).squeeze(1)
        w = row_weight if row_weight is not None else torch.full_like(rl, 1.0 / x.shape[0])
        return (rl * w).sum()

    @staticmethod
    def backward(ctx, dloss):
        x, y, row_weight, *params = ctx.saved_tensors
        L = ctx.nlayers
        Ws, bs = params[:L], params[L:]
        if ctx.native:
            dims = [Ws[0].shape[1]] + [W.shape[0] for W in Ws]
            dl = dloss.reshape(1).float().contiguous()
            _native.C().mlp(1, x.data_ptr(), y.data_ptr(), _native.ptr(row_weight), x.shape[0], dims,
                            [W.data_ptr() for W in Ws], [b.data_ptr() for b in bs],
                            [grad_buf(W).data_ptr() for W in Ws], [grad_buf(b).data_ptr() for b in bs], 0, 0,
                            dl.data_ptr(), ctx.act, _native.stream())
        else:
            with torch.enable_grad():
                ps = [p.detach().float().requires_grad_() for p in params]
                z = _ref_logits(x, ps[:L], ps[L:], ctx.act)
                rl = torch.logsumexp(z, 1) - z.gather(1, y[:, None]).squeeze(1)
                w = row_weight if row_weight is not None else torch.full_like(rl, 1.0 / x.shape[0])
                loss = (rl * w).sum()
                gs = torch.autograd.grad(loss, ps, dloss)
            for p, g in zip(params, gs):
                grad_buf(p).add_(g)
        grad_ready(*params)
        return (None,) * (5 + len(params))


def mlp_loss(x, y, weights, biases, act="sigmoid", row_weight=None):
    """Weighted-mean softmax CE of an MLP (weights in torch [out,in] layout)."""
    a = ACT[act] if isinstance(act, str) else act
    return MLPLossFn.apply(x, y, row_weight, a, len(weights), *weights, *biases)


def mlp_logits(x, weights, biases, act="sigmoid"):
    """Inference logits [n, C] (fused kernel on GPU)."""
    a = ACT[act] if isinstance(act, str) else act
    if _native.use_native(x):
        x = x.float().contiguous()
        C = weights[-1].shape[0]
        out = torch.empty(x.shape[0], C, device=x.device, dtype=torch.float32)
        dims = [weights[0].shape[1]] + [W.shape[0] for W in weights]
        _native.C().mlp(0, x.data_ptr(), 0, 0, x.shape[0], dims, [W.data_ptr() for W in weights],
                        [b.data_ptr() for b in biases], [], [], out.data_ptr(), 0, 0, a, _native.stream())
        return out
    with torch.no_grad():
        return _ref_logits(x, weights, biases, a)
