"""bf16 split planes of fp32 tensors: the operand format of the reference-precision GEMM.

An fp32 matrix X [R, C] is carried as a bf16 tensor P [3, R, ld] with X = P[0] + P[1] + P[2]
exactly (hi, mid, lo: each plane the round-to-nearest-even bf16 of what the planes before it
left), so a product of two fp32 values is the sum of six exact bf16 products
(csrc/include/smi_gemm_sp_impl.h).  Splitting costs VALU work; done inside a GEMM's k-loop it
made the fp32 GEMMs issue-bound (docs/PERF_NOTES.md, round 2b), so sparkmi splits every
operand ONCE, where it is produced:
  * weights — by the optimizer kernel that updates them (FlatParams.weight_planes, Adam/SGD);
  * activations / gradients — by the producing kernel's epilogue where it has one (the FFN
    hidden GEMM, the dgrad of linear2), otherwise by one ``split3`` pass, cached on the tensor
    (``_smi_planes``, valid while the tensor's version counter is unchanged) so that the forward
    GEMM and the weight-gradient GEMM that read the same activation share it.
A k-contiguous GEMM operand whose k extent is not a multiple of 32 (the vocabulary dimension in
the vocab projection's dgrad) is stored with ``ld`` rounded up and zero padding.
"""
import os

import torch

from .. import _native

# Planes-only gradients: a gradient whose every consumer reads split planes (the dY operand of a
# dgrad / wgrad GEMM pair) is written by its producer as planes alone — its fp32 tensor is a
# placeholder that is never filled unless a fallback path asks for it (f32() below).  The FFN
# hidden gradient, dlogits, the LayerNorm dh and the attention dQ/dK/dV skip 4 B per element.
PLANES_ONLY = True  # False (tests): every gradient also written in fp32


def r32(n):
    return (n + 31) // 32 * 32


def attach(t, planes):
    """Record ``planes`` as the split of ``t`` (valid until ``t`` is modified in place)."""
    t._smi_planes = (planes, t._version)
    return t


def cached(t, kpad=False):
    e = getattr(t, "_smi_planes", None)
    if e is None:
        # a reshape view of a tensor the producer split (shares its storage and version counter)
        b = t._base
        if b is not None and b.data_ptr() == t.data_ptr() and b.numel() == t.numel() and b.is_contiguous() \
                and t.is_contiguous():
            e = getattr(b, "_smi_planes", None)
    if e is None or e[1] != t._version:
        return None
    p = e[0]
    if kpad and p.stride(1) < r32(t.shape[-1]):
        return None
    return p


def new(rows, cols, device, kpad=False):
    """Uninitialised planes [3, rows, ld] (ld = cols, or cols rounded up to 32 with ``kpad``)."""
    ld = r32(cols) if kpad else (cols + 7) // 8 * 8
    return torch.empty(3, rows, ld, device=device, dtype=torch.bfloat16)


def split(t2, kpad=False, out=None):
    """Planes of a 2-D fp32 tensor (one split3 launch; padding columns zeroed)."""
    rows, cols = t2.shape
    P = out if out is not None else new(rows, cols, t2.device, kpad or cols % 8 != 0)
    _native.C().split3(t2.data_ptr(), rows, cols, t2.stride(0), P.data_ptr(), P.stride(1), P.stride(0),
                       _native.stream())
    return P


def of(t2, kpad=False):
    """The planes of a 2-D fp32 tensor: the producer's (cached) or a fresh split, cached."""
    p = cached(t2, kpad)
    if p is None:
        p = split(t2, kpad)
        attach(t2, p)
    return p


def weight(w):
    """Planes [3, N, K] of a weight: the optimizer-maintained flat planes when the parameter
    lives in a FlatParams buffer (FlatParams.weight_planes), else a fresh split (a parameter
    updated through its data pointer does not bump its version, so no cache here)."""
    fn = getattr(w, "_smi_planes_fn", None)
    if fn is not None:
        return fn()
    return split(w.detach().reshape(w.shape[0], -1))


def placeholder(like_shape, planes, device):
    """An fp32 tensor standing for the values held in ``planes`` (not filled: planes-only)."""
    t = torch.empty(like_shape, device=device, dtype=torch.float32)
    attach(t, planes)
    t._smi_planes_only = True
    return t


def mark_grad_planes_ok(t):
    """Declare that t's gradient may be planes-only: t was produced by a sparkmi Linear / FFN
    (whose backward reads dY through planes) and has exactly ONE differentiable consumer (autograd
    would otherwise add a second gradient to the placeholder).  The model code marks such tensors
    (sparkmi/models/transformer.py); user tensors are never marked, so a .grad stays real."""
    if t.dtype == torch.float32 and t.is_cuda:
        t._smi_gplanes = True
    return t


def grad_planes_ok(t):
    """A planes-only gradient for t is allowed: PLANES_ONLY is on and t came from a producer that
    reads planes (never a user tensor, whose .grad must hold real values)."""
    return PLANES_ONLY and any(b is not None and getattr(b, "_smi_gplanes", False) for b in (t, t._base))


def planes_only(t):
    """True when t (or the tensor t is a view of) holds its values in planes only."""
    return any(b is not None and getattr(b, "_smi_planes_only", False) for b in (t, t._base))


def f32(t):
    """Fill a planes-only tensor's fp32 values from its planes (hi + mid + lo, exact) so that a
    path that reads fp32 sees them; a no-op for ordinary tensors.  Returns t."""
    for b in (t, t._base):
        if b is None or not getattr(b, "_smi_planes_only", False):
            continue
        p = cached(b)
        if p is None:
            raise RuntimeError("planes-only tensor lost its planes")
        W = b.shape[-1]
        b2 = b.view(-1, W)
        torch.add(p[0, :, :W].float(), p[1, :, :W].float(), out=b2)
        b2.add_(p[2, :, :W].float())
        b._smi_planes_only = False
        attach(b, p)
    return t
