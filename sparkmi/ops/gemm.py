"""Python front-end of the MFMA GEMM (csrc/kernels/gemm.hip).

Three entry points, one per GEMM of a linear layer, each with its fused epilogue:
  fwd(x, w)        -> y = dropout(act(x @ w^T + bias))               bf16 out
  dgrad(dy, w)     -> dx = (dy @ w) [+ resid] [* relu'/dropout mask]  bf16 out
  wgrad(dy, x, gw) -> gw += dy^T @ x                                  fp32 accumulate (split-K)
``supported(...)`` says whether a shape can run on the kernel (K multiple of 64, dims multiple
of 8, 16-B aligned rows); other shapes run on the fp32 kernel (csrc/kernels/gemm_f32.hip, K % 4)
with upcast operands.  Every GEMM of the training step is one of these two hand-written kernels
(no vendor-library dispatch).
"""
import os

import torch

from .. import _native
from . import _grad

_DISABLE = False  # True (tests): every Linear on torch ops
NUM_CU = 256


def _aligned(*ts):
    return all(t is None or (t.data_ptr() % 16 == 0) for t in ts)


def supported(M, N, K, *tensors, mode=0):
    if _DISABLE:
        return False
    if K % 8 or K < 64 or M < 8 or N < 8:
        return False
    if mode != 0 and (M % 8 or N % 8):
        return False
    for t in tensors:
        if t is not None and (t.stride(-1) != 1 or (t.dim() > 1 and t.stride(-2) % 8)):
            return False
    return _aligned(*tensors)


def fwd(x, w, bias=None, act=0, rng=None, salt=0, thresh=0, dscale=1.0, out=None):
    M, K = x.shape
    N = w.shape[0]
    y = out if out is not None else torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    _native.C().gemm(0, x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), M, N, K, y.data_ptr(), y.stride(0), 0, 0,
                     0, 1.0, _native.ptr(bias), 0, 0, act, 0, 0, rng.ptr() if rng is not None else 0, salt, thresh,
                     dscale, 1, _native.stream())
    return y


def dgrad(dy, w, resid=None, dact_y=None, dscale=1.0, out=None):
    M, N = dy.shape
    K = w.shape[1]
    dx = out if out is not None else torch.empty(M, K, device=dy.device, dtype=torch.bfloat16)
    _native.C().gemm(1, dy.data_ptr(), dy.stride(0), w.data_ptr(), w.stride(0), M, K, N, dx.data_ptr(), dx.stride(0),
                     0, 0, 0, 1.0, 0, _native.ptr(resid), resid.stride(0) if resid is not None else 0, 0,
                     _native.ptr(dact_y), dact_y.stride(0) if dact_y is not None else 0, 0, 0, 0, dscale, 1,
                     _native.stream())
    return dx


# split-K target (workgroups) for the weight-gradient GEMM: it runs on the side stream next to
# the backward's critical path, so it need not fill the chip alone; fewer splits = fewer fp32
# atomic partial sums (each split adds one full N x K slab).
_WGRAD_TARGET = NUM_CU


def wgrad_splits(N, K, M):
    tiles = ((N + 127) // 128) * ((K + 127) // 128)
    s = 1
    while tiles * s < _WGRAD_TARGET and (M // (s * 2)) >= 256:
        s *= 2
    return s


_WGRAD_MODE = "slab"  # slab | atomic (tests)


def _actual_splits(M, s):
    """The split count the launcher really uses (k_per_split rounded up to the 64-deep k-step)."""
    kps = max(64, (M // s + 63) // 64 * 64)
    return (M + kps - 1) // kps


def wgrad(dy, x, gw, splits=None, gb=None, ready=None):
    """gw [N,K] fp32 += dy[M,N]^T @ x[M,K]; with ``gb`` also gb[N] += column sums of dy (the bias
    gradient, computed inside the same kernel by an extra MFMA per dy fragment).

    Split-K over M.  Slab mode (default): every split writes its partial tile to an fp32 slab
    with plain stores and one vectorised pass folds the slabs into ``gw`` — deterministic, and
    cheaper than fp32 atomics (which serialise at ~1.3 TB/s chip-wide: 16 splits of a 512x512
    gradient = 16 MB of atomic traffic).  Atomic mode accumulates straight into ``gw``.

    ``ready`` (the parameters whose gradients this completes): when given, the slab fold is
    queued (sparkmi/ops/_grad.py: one batched fold launch at the end of the backward, which then
    reports ``ready`` final) and True is returned; the caller must not report them itself."""
    M, N = dy.shape
    K = x.shape[1]
    s = splits or wgrad_splits(N, K, M)
    C = _native.C()
    if _WGRAD_MODE == "slab" and s > 1:
        s = _actual_splits(M, s)
        slab = torch.empty(s * N * K + (s * N if gb is not None else 0), device=gw.device, dtype=torch.float32)
        bslab = slab[s * N * K:] if gb is not None else None
        C.gemm_wgrad_slab(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), N, K, M, slab.data_ptr(), s,
                          _native.ptr(bslab), _native.stream())
        if ready is not None and _grad.FOLD_DEFER:
            _grad.defer_wgrad_fold(slab, s, N * K, gw, N if gb is not None else 0, gb, ready, _native.stream())
            return True
        C.splitk_reduce(slab.data_ptr(), s, N * K, gw.data_ptr(), N if gb is not None else 0, _native.ptr(gb), 1,
                        _native.stream())
        return gw
    C.gemm_wgrad_atomic(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), N, K, M, gw.data_ptr(),
                        gw.stride(0), s, _native.ptr(gb), _native.stream())
    return gw

# ---- fp32 (reference-precision) GEMM: csrc/kernels/gemm_f32.hip on v_mfma_f32_32x32x2_f32 ----
def supported32(M, N, K, *tensors, mode=0):
    """fp32 GEMM preconditions: float4 granularity along each operand's contiguous dimension
    (mode 0/1: K % 4; mode 1: N % 4; mode 2: the two output dims % 4), 16-B aligned rows."""
    if _DISABLE or M < 1 or N < 1 or K < 1:
        return False
    if mode in (0, 1) and K % 4:
        return False
    if mode in (1, 2) and N % 4:
        return False
    if mode == 2 and M % 4:
        return False
    for t in tensors:
        if t is not None and (t.dtype != torch.float32 or t.stride(-1) != 1 or (t.dim() > 1 and t.stride(-2) % 4)):
            return False
    return _aligned(*tensors)


def fwd32(x, w, bias=None, act=0, rng=None, salt=0, thresh=0, dscale=1.0, out=None):
    """y[M,N] = dropout(act(x[M,K] @ w[N,K]^T + bias)), fp32 in / out; act 0 none, 1 relu, 2 sigmoid."""
    M, K = x.shape
    N = w.shape[0]
    y = out if out is not None else torch.empty(M, N, device=x.device, dtype=torch.float32)
    _native.C().gemm_f32(0, x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), M, N, K, y.data_ptr(), y.stride(0),
                         0, 0, _native.ptr(bias), int(act), 0, 0, 0, 0,
                         rng.ptr() if rng is not None else 0, salt, thresh, dscale, 1, 0, _native.stream())
    return y


def dgrad32(dy, w, resid=None, dact_y=None, dscale=1.0, out=None):
    """dx[M,K] = (dy[M,N] @ w[N,K]) (+ resid) (* [dact_y > 0] * dscale), fp32."""
    M, N = dy.shape
    K = w.shape[1]
    dx = out if out is not None else torch.empty(M, K, device=dy.device, dtype=torch.float32)
    _native.C().gemm_f32(1, dy.data_ptr(), dy.stride(0), w.data_ptr(), w.stride(0), M, K, N, dx.data_ptr(),
                         dx.stride(0), 0, 0, 0, 0, _native.ptr(resid), resid.stride(0) if resid is not None else 0,
                         _native.ptr(dact_y), dact_y.stride(0) if dact_y is not None else 0, 0, 0, 0, dscale, 1, 0,
                         _native.stream())
    return dx


def wgrad32(dy, x, gw, gb=None, splits=None):
    """gw[N,K] += dy[M,N]^T @ x[M,K] (and gb[N] += column sums of dy), fp32.  Standalone form:
    split-K over the M tokens with fp32 atomics so a few output tiles still fill the chip (the
    training path queues wgrads into one grouped launch instead, sparkmi/ops/_grad.py)."""
    M, N = dy.shape
    K = x.shape[1]
    tiles = ((N + 127) // 128) * ((K + 127) // 128)
    s = splits or max(1, min(M // 256, (2 * NUM_CU + tiles - 1) // tiles))
    _native.C().gemm_f32(2, dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), N, K, M, gw.data_ptr(),
                         gw.stride(0), 1, int(s > 1), 0, 0, 0, 0, 0, 0, 0, 0, 0, 1.0, s, _native.ptr(gb),
                         _native.stream())
    return gw


# ---- split-plane fp32 GEMM: csrc/kernels/gemm_sp*.hip (operands as bf16 hi/mid/lo planes) ----
# The reference-precision path of the fp32 Linear layers (sparkmi/ops/planes.py): six exact bf16
# slice products per fp32 product on v_mfma_f32_32x32x16_bf16, no splitting inside the k-loop.
# SP = False falls back to csrc/kernels/gemm_f32.hip (split inside the GEMM; the bench's f32-MFMA
# comparison run).
SP = not _DISABLE


def _sp_ok(*ts):
    return all(t is None or (t.dtype == torch.float32 and t.stride(-1) == 1 and t.data_ptr() % 16 == 0
                             and (t.dim() < 2 or t.stride(-2) % 4 == 0)) for t in ts)


def sp_fwd(xp, wp, M, N, K, bias=None, act=0, rng=None, salt=0, thresh=0, dscale=1.0, out_planes=False, mask=None):
    """y[M,N] = dropout(act(x @ w^T + bias)) from planes xp [3,M,>=K], wp [3,N,>=K].  Returns
    (y, y_planes or None), or None when the kernel does not cover the case (caller falls back).
    ``mask``: uint8 [M, ceil(N/4)] receiving bit e of column group c = (y[:, 4c + e] > 0) INSTEAD
    of the fp32 y (returned None; planes required) — the FFN hidden activation's sign for the
    linear2 dgrad epilogue."""
    if not SP or act not in (0, 1) or not _sp_ok(bias):
        return None
    if mask is not None and not (out_planes and N % 32 == 0):
        return None
    y = torch.empty(M, N, device=xp.device, dtype=torch.float32) if mask is None else None
    yp = None
    if out_planes and N % 32 == 0:
        yp = torch.empty(3, M, N, device=xp.device, dtype=torch.bfloat16)
    ok = _native.C().gemm_sp(0, xp.data_ptr(), xp.stride(1), xp.stride(0), wp.data_ptr(), wp.stride(1), wp.stride(0),
                             # ldc = N without an fp32 output: the dropout hash index is row * ldc + col
                             M, N, K, 0, _native.ptr(y), y.stride(0) if y is not None else N, _native.ptr(yp), N,
                             yp.stride(0) if yp is not None else 0, 0, _native.ptr(bias), int(act), 0, 0, 0, 0,
                             rng.ptr() if rng is not None else 0, salt, thresh, dscale, 0, _native.ptr(mask), mask.stride(0) if mask is not None else 0, _native.stream())
    return (y, yp) if ok else None


def sp_dgrad(dyp, wp, M, K, N, resid=None, dact_y=None, dscale=1.0, out_planes=False, need_f32=True, dmask=None):
    """dx[M,K] = (dy @ w) (+ resid) (* [dact_y > 0] dscale) from planes dyp [3,M,>=N] (zero-padded
    to a multiple of 32 when N is not), wp [3,N,K].  ``dmask`` (uint8 [M, ceil(K/4)], sp_fwd's
    ``mask``) stands in for dact_y.  Returns (dx or None, dx_planes or None)."""
    if not SP or not _sp_ok(resid, dact_y) or (dmask is not None and dact_y is not None):
        return None
    dx = torch.empty(M, K, device=dyp.device, dtype=torch.float32) if need_f32 else None
    dxp = None
    if out_planes and K % 32 == 0:
        dxp = torch.empty(3, M, K, device=dyp.device, dtype=torch.bfloat16)
    if dx is None and dxp is None:
        return None
    ok = _native.C().gemm_sp(1, dyp.data_ptr(), dyp.stride(1), dyp.stride(0), wp.data_ptr(), wp.stride(1),
                             wp.stride(0), M, K, N, int(dyp.stride(1) >= (N + 31) // 32 * 32), _native.ptr(dx),
                             dx.stride(0) if dx is not None else K, _native.ptr(dxp), K,
                             dxp.stride(0) if dxp is not None else 0, 0, 0, 0, _native.ptr(resid),
                             resid.stride(0) if resid is not None else 0, _native.ptr(dact_y),
                             dact_y.stride(0) if dact_y is not None else 0, 0, 0, 0, dscale, 0,
                             _native.ptr(dmask), dmask.stride(0) if dmask is not None else 0, _native.stream())
    return (dx, dxp) if ok else None


def sp_wgrad(dyp, xp, gw, gb=None):
    """gw[N,K] += dy^T x (and gb[N] += colsum dy) from planes dyp [3,M,>=N], xp [3,M,>=K]; one
    launch, full token reduction per tile.  Returns False when not covered."""
    if not SP or not gw.is_contiguous() or (gb is not None and not gb.is_contiguous()):
        return False
    N, K = gw.shape
    M = dyp.shape[1]
    return bool(_native.C().gemm_sp(2, dyp.data_ptr(), dyp.stride(1), dyp.stride(0), xp.data_ptr(), xp.stride(1),
                                    xp.stride(0), N, K, M, 0, gw.data_ptr(), gw.stride(0), 0, 0, 0, 1, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 1.0, _native.ptr(gb), 0, 0, _native.stream()))
