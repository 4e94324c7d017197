"""Fused FashionMNIST-CNN training op (csrc/kernels/cnn.hip).

``cnn_loss(x, y, params)`` = mean cross-entropy of the reference CNN (distributed_cnn.py:47-86)
over the batch.  GPU: ONE kernel launch runs forward AND backward for every image (one
workgroup per image, activations in LDS) and leaves per-image gradients in a slab (the conv
layers' gradients, then the image's logit gradient dl and pooled activations p2: the fc
gradient is their outer product, formed by the reducer); the autograd backward is one reduce
launch that sums the slab over images, scales by dloss and accumulates into the parameters' (flat) fp32 gradients.  CPU: the identical math with torch
(conv2d / max_pool2d / linear), so the kernel is testable against it.
"""
import torch
import torch.nn.functional as F

from .. import _native
from ._grad import grad_buf, grad_ready


def reference_logits(x, params, x_scale=None):
    """Torch reference of the reference model's forward (NCHW)."""
    w1, b1, w2, b2, w3, b3, w4, b4, wf, bf = params
    if x.dtype == torch.uint8:
        x = x.float() * (x_scale if x_scale is not None else 1.0 / 255.0)
    h = F.relu(F.conv2d(x.float(), w1, b1, padding=1))
    h = F.relu(F.conv2d(h, w2, b2, padding=1))
    h = F.max_pool2d(h, 2)
    h = F.relu(F.conv2d(h, w3, b3, padding=1))
    h = F.relu(F.conv2d(h, w4, b4, padding=1))
    h = F.max_pool2d(h, 2)
    return F.linear(h.flatten(1), wf, bf)


def _launch(phase, x, y, params, grads, slab, row_loss, pred, logits, loss, loss_scale, dloss, train, bf16=False):
    w = [params[i] for i in (0, 2, 4, 6, 8)]
    b = [params[i] for i in (1, 3, 5, 7, 9)]
    B, cin = x.shape[0], x.shape[1]
    C, classes = w[0].shape[0], w[4].shape[0]
    gw = [grads[i].data_ptr() for i in (0, 2, 4, 6, 8)] if grads else []
    gb = [grads[i].data_ptr() for i in (1, 3, 5, 7, 9)] if grads else []
    _native.C().cnn(phase, x.data_ptr(), int(x.dtype == torch.uint8), 1.0 / 255.0, _native.ptr(y), B, cin, C, classes,
                    [t.data_ptr() for t in w], [t.data_ptr() for t in b], gw, gb, _native.ptr(slab),
                    _native.ptr(row_loss), _native.ptr(pred), _native.ptr(logits), _native.ptr(loss), loss_scale,
                    _native.ptr(dloss), int(train), int(bf16), _native.stream())


def num_params(params):
    return sum(p.numel() for p in params)


class CNNLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y, bf16, *params):
        ctx.native = _native.use_native(x)
        B = x.shape[0]
        if ctx.native:
            x = x.contiguous()
            y = y.to(torch.int64).contiguous()
            params = [p.contiguous() for p in params]
            slab = torch.empty(B, num_params(params), device=x.device, dtype=torch.float32)
            row_loss = torch.empty(B, device=x.device, dtype=torch.float32)
            pred = torch.empty(B, device=x.device, dtype=torch.int32)
            loss = torch.empty(1, device=x.device, dtype=torch.float32)
            _launch(0, x, y, params, None, slab, row_loss, pred, None, loss, 1.0 / B, None, True, bf16)
            ctx.save_for_backward(slab, *params)
            ctx.pred = pred
            return loss[0]
        ctx.save_for_backward(x, y, *params)
        with torch.no_grad():
            z = reference_logits(x, [p.float() for p in params])
            return F.cross_entropy(z, y)

    @staticmethod
    def backward(ctx, dloss):
        if ctx.native:
            slab, *params = ctx.saved_tensors
            grads = [grad_buf(p) for p in params]
            dl = dloss.reshape(1).float().contiguous()
            x_dummy = slab  # only its shape is unused in phase 1
            w = [params[i] for i in (0, 2, 4, 6, 8)]
            _native.C().cnn(1, 0, 0, 0.0, 0, slab.shape[0], w[0].shape[1], w[0].shape[0], w[4].shape[0],
                            [t.data_ptr() for t in w], [params[i].data_ptr() for i in (1, 3, 5, 7, 9)],
                            [grads[i].data_ptr() for i in (0, 2, 4, 6, 8)],
                            [grads[i].data_ptr() for i in (1, 3, 5, 7, 9)], slab.data_ptr(), 0, 0, 0, 0, 0.0,
                            dl.data_ptr(), 1, 0, _native.stream())
            del x_dummy
        else:
            x, y, *params = ctx.saved_tensors
            with torch.enable_grad():
                ps = [p.detach().float().requires_grad_() for p in params]
                loss = F.cross_entropy(reference_logits(x, ps), y)
                gs = torch.autograd.grad(loss, ps, dloss)
            for p, g in zip(params, gs):
                grad_buf(p).add_(g)
        grad_ready(*params)
        return (None, None, None) + (None,) * len(params)


def cnn_loss(x, y, params, bf16=False):
    """Mean CE of the fused CNN step; ``bf16``: the convolutions run on bf16 matrix cores
    (fp32 accumulation and fp32 activations / gradients elsewhere) on the GPU."""
    return CNNLossFn.apply(x, y, bool(bf16), *params)


def cnn_logits(x, params, bf16=False):
    if _native.use_native(x):
        x = x.contiguous()
        B = x.shape[0]
        logits = torch.empty(B, params[8].shape[0], device=x.device, dtype=torch.float32)
        _launch(0, x, None, [p.contiguous() for p in params], None, None, None, None, logits, None, 1.0, None, False,
                bf16)
        return logits
    with torch.no_grad():
        return reference_logits(x, [p.float() for p in params])


# the conv4 / conv3 / conv2 weight gradients on helper workgroups beside the image's dgrad chain
# (csrc/kernels/cnn.hip cnn_wgrad_helper; fused steps)
WGRAD_HELPERS = True


def _hand(B, C, device):
    """The helpers' hand-off area ([B][cnn_hand_floats(C)] floats) or None (helpers off)."""
    n = _native.C().cnn_hand_floats(C) if WGRAD_HELPERS else 0
    return torch.empty(B * n, device=device, dtype=torch.float32) if n else None


def cnn_sgd_step(x, y, params, lr_t, step_t, tick, shadows=None, bf16=False, index=None):
    """The whole training step — forward, mean CE, backward, gradient reduction over the batch
    and the SGD update — as ONE launch (csrc/kernels/cnn.hip, CNNArgs::fused): the per-image
    slabs are summed in the kernel's ticketed tail, which then updates ``params`` in place
    (p -= lr * g; ``lr_t`` / ``step_t`` are the optimizer's device scalars) and their bf16
    ``shadows`` (10 tensors or None).  Returns the step's mean loss (device scalar).  ``tick``:
    CNN_TICKS + 3 B zeroed int32 counters owned by the model (the kernel re-arms them).
    ``index`` = (batch, perm, cursor): ``x`` / ``y`` are the whole dataset and the kernel reads image
    i of the batch from row perm[cursor * batch + i], then advances the device cursor (the shuffled
    batch gather inside the step kernel; DeviceLoader fixed=True, index mode)."""
    B = index[0] if index is not None else x.shape[0]
    w = [params[i] for i in (0, 2, 4, 6, 8)]
    b = [params[i] for i in (1, 3, 5, 7, 9)]
    P = num_params(params)
    slab = torch.empty(B, P, device=x.device, dtype=torch.float32)
    row_loss = torch.empty(B, device=x.device, dtype=torch.float32)
    loss = torch.empty(1, device=x.device, dtype=torch.float32)
    _native.C().cnn_sgd_step(x.data_ptr(), int(x.dtype == torch.uint8), 1.0 / 255.0, y.data_ptr(), B, x.shape[1],
                             w[0].shape[0], w[4].shape[0], [t.data_ptr() for t in w], [t.data_ptr() for t in b],
                             [t.data_ptr() for t in shadows] if shadows else [], slab.data_ptr(),
                             row_loss.data_ptr(), loss.data_ptr(), 1.0 / B, lr_t.data_ptr(), step_t.data_ptr(),
                             tick.data_ptr(), int(bf16), index[1].data_ptr() if index else 0,
                             index[2].data_ptr() if index else 0, _native.ptr(_hand(B, w[0].shape[0], x.device)),
                             _native.stream())
    return loss[0]


def cnn_grad_step(x, y, params, grads, tick, bf16=False, index=None):
    """Forward, mean CE, backward and the gradient reduction over the batch as ONE launch, the
    batch gradient ADDED to ``grads`` (10 fp32 tensors: the flat gradient buffer's slices) — the
    data-parallel step's local half (csrc/kernels/cnn.hip gradient mode): the executors'
    gradients are then all-reduced and the optimizer applies them.  Returns the mean loss.
    ``index``: as in cnn_sgd_step."""
    B = index[0] if index is not None else x.shape[0]
    w = [params[i] for i in (0, 2, 4, 6, 8)]
    b = [params[i] for i in (1, 3, 5, 7, 9)]
    P = num_params(params)
    slab = torch.empty(B, P, device=x.device, dtype=torch.float32)
    row_loss = torch.empty(B, device=x.device, dtype=torch.float32)
    loss = torch.empty(1, device=x.device, dtype=torch.float32)
    _native.C().cnn_grad_step(x.data_ptr(), int(x.dtype == torch.uint8), 1.0 / 255.0, y.data_ptr(), B, x.shape[1],
                              w[0].shape[0], w[4].shape[0], [t.data_ptr() for t in w], [t.data_ptr() for t in b],
                              [grads[i].data_ptr() for i in (0, 2, 4, 6, 8)],
                              [grads[i].data_ptr() for i in (1, 3, 5, 7, 9)], slab.data_ptr(),
                              row_loss.data_ptr(), loss.data_ptr(), 1.0 / B, tick.data_ptr(), int(bf16),
                              index[1].data_ptr() if index else 0, index[2].data_ptr() if index else 0,
                              _native.ptr(_hand(B, w[0].shape[0], x.device)), _native.stream())
    return loss[0]
