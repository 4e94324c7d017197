"""Parameter-gradient plumbing shared by every fused op.

sparkmi's fused autograd Functions do not hand weight gradients back to autograd; their
backward kernels accumulate them straight into ``param.grad`` (an fp32 view into the model's
flat gradient buffer when the model was flattened by :class:`sparkmi.utils.flat.FlatParams`),
then call :func:`grad_ready` so the data-parallel engine can launch the all-reduce of a
gradient bucket as soon as its last parameter is final (overlap with the rest of backward).
"""
import torch

_listeners = []


def add_listener(fn):
    _listeners.append(fn)
    return fn


def remove_listener(fn):
    if fn in _listeners:
        _listeners.remove(fn)


def grad_buf(p: torch.Tensor) -> torch.Tensor:
    """fp32 gradient accumulator of parameter ``p`` (allocated lazily when not flattened)."""
    if p.grad is None:
        p.grad = torch.zeros_like(p, dtype=torch.float32)
    return p.grad


def accumulate(p: torch.Tensor, g: torch.Tensor):
    """p.grad += g (fp32)."""
    buf = grad_buf(p)
    buf.add_(g.reshape(buf.shape).to(buf.dtype))


def grad_ready(*params):
    for fn in _listeners:
        for p in params:
            if p is not None:
                fn(p)


def bf16_weight(p: torch.Tensor) -> torch.Tensor:
    """bf16 compute copy of a master fp32 parameter (flat shadow when available)."""
    w = getattr(p, "_smi_bf16", None)
    if w is not None:
        return w
    return p.detach().to(torch.bfloat16)


def needs_input_grad(ctx, i):
    return ctx.needs_input_grad[i]
