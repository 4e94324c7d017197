"""Fused small-MLP (affine + sigmoid/relu hidden layers + affine logits + softmax-CE).

One HIP launch computes the (weighted) mean cross-entropy of a whole minibatch or full batch;
one launch recomputes the forward and accumulates every weight/bias gradient; and
``mlp_sgd_step`` is a whole training step (forward, CE, backward, SGD update) in ONE launch
(csrc/kernels/mlp.hip).  Cross-block sums are deterministic (block-order reduction).  Used by the reference MLP (distributed_multilayer_perceptron.py:44-53)
and by the MLlib-compatible MultilayerPerceptronClassifier's L-BFGS objective.
``row_weight`` implements MLlib's per-block loss averaging.
"""
import torch

from .. import _native
from ._grad import grad_buf, grad_ready

ACT = {"sigmoid": 2, "relu": 1}
_ws = {}


def _workspace(device, n, dims):
    """(ws, ticket) device pointers for the kernel's cross-block reduction (0, 0 for one block).
    Cached per (device, size) and never freed: captured graphs keep using the same buffers."""
    grid = _native.C().mlp_grid(int(n))
    if grid <= 1:
        return 0, 0
    T = sum(dims[i + 1] * (dims[i] + 1) for i in range(len(dims) - 1))
    key = (str(device), grid * (T + 1))
    e = _ws.get(key)
    if e is None:
        e = _ws[key] = (torch.empty(grid * (T + 1), device=device, dtype=torch.float32),
                        torch.zeros(1, device=device, dtype=torch.int32))
    return e[0].data_ptr(), e[1].data_ptr()


def _dims(Ws):
    return [Ws[0].shape[1]] + [W.shape[0] for W in Ws]


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
            dims = _dims(Ws)
            ws, tk = _workspace(x.device, x.shape[0], dims)
            _native.C().mlp(0, x.data_ptr(), y.data_ptr(), _native.ptr(row_weight), x.shape[0], dims,
                            [W.data_ptr() for W in Ws], [b.data_ptr() for b in bs], [], [], 0, loss.data_ptr(), 0,
                            act, ws, tk, 0, 0, 0, 1.0, _native.stream())
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
            dims = _dims(Ws)
            dl = dloss.reshape(1).float().contiguous()
            ws, tk = _workspace(x.device, x.shape[0], dims)
            _native.C().mlp(1, x.data_ptr(), y.data_ptr(), _native.ptr(row_weight), x.shape[0], dims,
                            [W.data_ptr() for W in Ws], [b.data_ptr() for b in bs],
                            [grad_buf(W).data_ptr() for W in Ws], [grad_buf(b).data_ptr() for b in bs], 0, 0,
                            dl.data_ptr(), ctx.act, ws, tk, 1, 0, 0, 1.0, _native.stream())
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


def mlp_sgd_step(x, y, weights, biases, lr_t, step_t=None, act="sigmoid", row_weight=None, grad_scale=1.0,
                 loss_out=None):
    """One training step in ONE launch: forward, weighted softmax-CE, backward and plain SGD
    (params -= lr * grad_scale * grad, ``step_t`` += 1) on the GPU.  Parameters must be fp32
    contiguous device tensors (updated in place); ``lr_t`` a device scalar.  Returns the loss
    (device scalar) of the step's forward, i.e. before the update."""
    a = ACT[act] if isinstance(act, str) else act
    x = x.float().contiguous()
    y = y.to(torch.int64).contiguous()
    loss = loss_out if loss_out is not None else torch.empty(1, device=x.device, dtype=torch.float32)
    dims = _dims(weights)
    ws, tk = _workspace(x.device, x.shape[0], dims)
    _native.C().mlp(2, x.data_ptr(), y.data_ptr(), _native.ptr(row_weight), x.shape[0], dims,
                    [W.data_ptr() for W in weights], [b.data_ptr() for b in biases], [], [], 0, loss.data_ptr(), 0,
                    a, ws, tk, 0, lr_t.data_ptr(), _native.ptr(step_t), float(grad_scale), _native.stream())
    return loss[0]


def mlp_sgd_steps(batches, weights, biases, lr_t, step_t=None, act="sigmoid", grad_scale=1.0, index=None):
    """``len(batches)`` consecutive fused SGD steps (``mlp_sgd_step`` on each (x, y) in order) in
    ONE launch — the 4-5-4-3 kernel keeps the parameters on chip between steps, bitwise the same
    steps.  Returns the per-step losses (device scalars), or None when the shapes are not covered
    (the caller then runs one launch per step).  ``index`` = (batch, perm, cursor, steps): the
    batches are read from the dataset ``batches[0]`` = (x_all, y_all), step t's row i being
    perm[(cursor + t) * batch + i] (DeviceLoader fixed=True, index mode; cursor += steps)."""
    a = ACT[act] if isinstance(act, str) else act
    if index is not None:
        n, perm, cursor, nsteps = index
        batches = [batches[0]] * nsteps
    else:
        n, perm, cursor = batches[0][0].shape[0], None, None
    if any((index is None and x.shape[0] != n) or x.dtype != torch.float32 or not x.is_contiguous()
           or y.dtype != torch.int64 or not y.is_contiguous() for x, y in batches):
        return None
    # [step losses..., their sum in step order] (the sum: the runner's group total, no reduction launch)
    losses = torch.empty(len(batches) + 1, device=batches[0][0].device, dtype=torch.float32)
    ok = _native.C().mlp_steps([x.data_ptr() for x, _ in batches], [y.data_ptr() for _, y in batches],
                               [losses[i:].data_ptr() for i in range(len(batches))], n, _dims(weights),
                               [W.data_ptr() for W in weights], [b.data_ptr() for b in biases], a,
                               lr_t.data_ptr(), _native.ptr(step_t), float(grad_scale), _native.ptr(perm),
                               _native.ptr(cursor), losses[len(batches):].data_ptr(), _native.stream())
    if not ok:
        return None
    out = StepLosses(losses[i] for i in range(len(batches)))
    out.total = losses[len(batches)]
    return out


class StepLosses(list):
    """Per-step losses of a multi-step launch; ``total``: their sum, written by the same kernel."""
    total = None


def mlp_grad_step(x, y, weights, biases, act="sigmoid", row_weight=None):
    """Forward, weighted softmax-CE and backward in ONE launch, the gradients ADDED to the
    parameters' (flat) gradient buffers — the data-parallel step's local half (the all-reduce and
    the optimizer follow).  Returns the loss (device scalar)."""
    a = ACT[act] if isinstance(act, str) else act
    x = x.float().contiguous()
    y = y.to(torch.int64).contiguous()
    loss = torch.empty(1, device=x.device, dtype=torch.float32)
    dims = _dims(weights)
    ws, tk = _workspace(x.device, x.shape[0], dims)
    _native.C().mlp(1, x.data_ptr(), y.data_ptr(), _native.ptr(row_weight), x.shape[0], dims,
                    [W.data_ptr() for W in weights], [b.data_ptr() for b in biases],
                    [grad_buf(W).data_ptr() for W in weights], [grad_buf(b).data_ptr() for b in biases], 0,
                    loss.data_ptr(), 0, a, ws, tk, 1, 0, 0, 1.0, _native.stream())
    return loss[0]


def mlp_logits(x, weights, biases, act="sigmoid"):
    """Inference logits [n, C] (fused kernel on GPU)."""
    a = ACT[act] if isinstance(act, str) else act
    if _native.use_native(x):
        x = x.float().contiguous()
        C = weights[-1].shape[0]
        out = torch.empty(x.shape[0], C, device=x.device, dtype=torch.float32)
        dims = [weights[0].shape[1]] + [W.shape[0] for W in weights]
        ws, tk = _workspace(x.device, x.shape[0], dims)
        _native.C().mlp(0, x.data_ptr(), 0, 0, x.shape[0], dims, [W.data_ptr() for W in weights],
                        [b.data_ptr() for b in biases], [], [], out.data_ptr(), 0, 0, a, ws, tk, 0, 0, 0, 1.0,
                        _native.stream())
        return out
    with torch.no_grad():
        return _ref_logits(x, weights, biases, a)
