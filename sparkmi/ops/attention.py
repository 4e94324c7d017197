"""Fused multi-head attention core (softmax(QK^T/sqrt(d) + bias) V) for head_dim 64.

Reads q/k/v directly out of the fused projection outputs in the reference's per-head
interleaved layouts and writes the head-merged output:
  * self-attention: qkv [B,S,H*3*hd] with head h = [q_h | k_h | v_h]  (transformer.py:74-81)
  * cross-attention: q [B,Sq,H*hd], kv [B,Sk,H*2*hd] with head h = [k_h | v_h]
    (transformer.py:177-190)

Mask modes (SURVEY.md Q6 — the reference's boolean-mask addition semantics):
  * "none"      — no mask (also what the reference's encoder padding mask reduces to);
  * "reference" — +1.0 added to the scores of strictly-past keys (the reference's
                  "look-ahead" mask after its permute; used for decoder self and cross attn);
  * "causal"    — true causal masking (-inf on future keys; upper tiles skipped);
  * key_padding — optional bool [B,Sk], -inf on padded keys (true padding masking).
GPU: csrc/kernels/attention.hip (bf16 activations, 16x16x32 bf16 MFMA) or
csrc/kernels/attention_f32.hip (fp32 activations = reference precision, 32x32x2 f32 MFMA); both
flash-style forward + dQ and dK/dV backward kernels, no S x S tensor in HBM.  CPU: torch
reference math in fp32.
"""
import math

import torch

from .. import _native
from . import planes as _pl

MODES = {"none": 0, None: 0, "reference": 1, "causal": 2}
_LOG2E = 1.4426950408889634


def _bias_mask(Sq, Sk, mode, key_padding, device, B):
    """Additive fp32 bias [B or 1, 1, Sq, Sk] for the reference path."""
    bias = torch.zeros(1, 1, Sq, Sk, device=device)
    qi = torch.arange(Sq, device=device)[:, None]
    kj = torch.arange(Sk, device=device)[None, :]
    if mode == 1:
        bias = bias + (kj < qi).float()
    elif mode == 2:
        bias = bias.masked_fill(kj > qi, float("-inf"))
    if key_padding is not None:
        bias = bias + torch.zeros(B, 1, 1, Sk, device=device).masked_fill(key_padding[:, None, None, :].bool(),
                                                                           float("-inf"))
    return bias


def attention_reference(q, k, v, mode=0, key_padding=None):
    """q [B,H,Sq,hd], k/v [B,H,Sk,hd] -> out [B,H,Sq,hd] (fp32 math)."""
    B, H, Sq, hd = q.shape
    Sk = k.shape[2]
    s = (q.float() @ k.float().transpose(-1, -2)) / math.sqrt(hd)
    s = s + _bias_mask(Sq, Sk, mode, key_padding, q.device, B)
    p = torch.softmax(s, dim=-1)
    p = torch.nan_to_num(p, nan=0.0)
    return p @ v.float()


def _split_self(qkv, H):
    B, S, F = qkv.shape
    hd = F // (3 * H)
    t = qkv.reshape(B, S, H, 3 * hd).permute(0, 2, 1, 3)
    return t[..., :hd], t[..., hd:2 * hd], t[..., 2 * hd:]


def _split_cross(q, kv, H):
    B, Sq, D = q.shape
    hd = D // H
    Sk = kv.shape[1]
    qh = q.reshape(B, Sq, H, hd).permute(0, 2, 1, 3)
    t = kv.reshape(B, Sk, H, 2 * hd).permute(0, 2, 1, 3)
    return qh, t[..., :hd], t[..., hd:]


def _merge(o):
    B, H, S, hd = o.shape
    return o.permute(0, 2, 1, 3).reshape(B, S, H * hd)


def _planes_like(t):
    """Planes [3, rows, W] for an fp32 [.., W] attention output / gradient (None: planes off or W
    not a multiple of 32, the split-plane GEMM's k granularity)."""
    from . import gemm as G
    W = t.shape[-1]
    if t.dtype != torch.float32 or not G.SP or W % 32 or not t.is_contiguous():
        return None
    return torch.empty(3, t.numel() // W, W, device=t.device, dtype=torch.bfloat16)


class _AttnCore(torch.autograd.Function):
    """Shared autograd core.  ``views`` describe (base tensor, offset, (sb, ss, sh)) for q/k/v."""

    @staticmethod
    def forward(ctx, qsrc, kvsrc, H, mode, key_padding, cross, kv_col=0, shared=None):
        ctx.H, ctx.mode, ctx.cross = H, mode, cross
        ctx.native = _native.use_native(qsrc)
        ctx.kv_col, ctx.shared = kv_col, shared
        if not ctx.native:
            if shared is not None or kv_col:
                raise ValueError("column-sliced kv with a shared gradient is a GPU-kernel path")
            if cross:
                qh, kh, vh = _split_cross(qsrc, kvsrc, H)
            else:
                qh, kh, vh = _split_self(qsrc, H)
            qh, kh, vh = qh.detach().requires_grad_(), kh.detach().requires_grad_(), vh.detach().requires_grad_()
            with torch.enable_grad():
                o = attention_reference(qh, kh, vh, mode, key_padding)
            ctx.ref = (qh, kh, vh, o)
            ctx.save_for_backward()
            return _merge(o.detach()).to(qsrc.dtype)
        C = _native.C()
        qsrc = qsrc.contiguous()
        f32 = qsrc.dtype == torch.float32
        es = qsrc.element_size()  # pointer offsets below are in bytes
        B, Sq = qsrc.shape[0], qsrc.shape[1]
        if cross:
            kvsrc = kvsrc.contiguous()
            if kvsrc.dtype != qsrc.dtype:
                raise TypeError(f"cross attention: q dtype {qsrc.dtype} != kv dtype {kvsrc.dtype}")
            hd = qsrc.shape[2] // H
            Sk, W = kvsrc.shape[1], kvsrc.shape[2]  # W: 2*H*hd, or the width of a concatenated kv
            if kv_col < 0 or kv_col + 2 * H * hd > W:
                raise ValueError(f"cross attention: kv columns [{kv_col}, {kv_col + 2 * H * hd}) outside width {W}")
            qp, qs = qsrc.data_ptr(), (Sq * H * hd, H * hd, hd)
            kp, ks = kvsrc.data_ptr() + kv_col * es, (Sk * W, W, 2 * hd)
            vp, vs = kp + hd * es, ks
        else:
            hd = qsrc.shape[2] // (3 * H)
            Sk = Sq
            qp, qs = qsrc.data_ptr(), (Sq * 3 * H * hd, 3 * H * hd, 3 * hd)
            kp, ks = qp + hd * es, qs
            vp, vs = qp + 2 * hd * es, qs
        if hd != 64:
            raise NotImplementedError("sparkmi attention kernel supports head_dim 64")
        o = torch.empty(B, Sq, H * hd, device=qsrc.device, dtype=qsrc.dtype if f32 else torch.bfloat16)
        lse = torch.empty(B, H, Sq, device=qsrc.device, dtype=torch.float32)
        os_ = (Sq * H * hd, H * hd, hd)
        kpad = key_padding.to(torch.uint8).contiguous() if key_padding is not None else None
        if f32:
            opl = _planes_like(o)  # the out-projection's operand, written by the same epilogue
            C.attn_f32_fwd(qp, kp, vp, qs, ks, vs, o.data_ptr(), os_, lse.data_ptr(), _native.ptr(kpad), B, H, Sq, Sk,
                           mode, _LOG2E / math.sqrt(hd), _native.ptr(opl), opl.stride(0) if opl is not None else 0,
                           _native.stream())
            if opl is not None:
                _pl.attach(o, opl)
        else:
            C.attn_fwd(qp, kp, vp, qs, ks, vs, o.data_ptr(), os_, lse.data_ptr(), _native.ptr(kpad), B, H, Sq, Sk, mode,
                       _LOG2E / math.sqrt(hd), _native.stream())
        ctx.geom = (B, Sq, Sk, hd, qs, ks, vs, os_)
        ctx.kpad = kpad
        ctx.save_for_backward(qsrc, kvsrc if cross else None, o, lse)
        return o

    @staticmethod
    def backward(ctx, do):
        if not ctx.native:
            qh, kh, vh, o = ctx.ref
            B, H, S, hd = o.shape
            do_h = do.float().reshape(B, S, H, hd).permute(0, 2, 1, 3)
            dq, dk, dv = torch.autograd.grad(o, (qh, kh, vh), do_h)
            if ctx.cross:
                dqs = _merge(dq)
                dkv = torch.cat([dk, dv], dim=-1).permute(0, 2, 1, 3).reshape(B, kh.shape[2], -1)
                return dqs.to(do.dtype), dkv.to(do.dtype), None, None, None, None, None, None
            dqkv = torch.cat([dq, dk, dv], dim=-1).permute(0, 2, 1, 3).reshape(B, S, -1)
            return dqkv.to(do.dtype), None, None, None, None, None, None, None
        C = _native.C()
        qsrc, kvsrc, o, lse = ctx.saved_tensors
        B, Sq, Sk, hd, qs, ks, vs, os_ = ctx.geom
        H = ctx.H
        do = do.contiguous()
        if do.dtype != o.dtype:
            do = do.to(o.dtype)
        es = qsrc.element_size()
        delta = torch.empty(B, H, Sq, device=do.device, dtype=torch.float32)
        f32 = qsrc.dtype == torch.float32
        # split planes of the gradients (fp32): the dY operands of the projections' dgrad / wgrad
        # GEMMs, at the same element offsets as the fp32 gradients (2 B per element per plane)
        pq = pk = pv = 0
        q_ps = kv_ps = 0
        if ctx.cross:
            dq = torch.empty_like(qsrc)
            dkv = ctx.shared.get(kvsrc) if ctx.shared is not None else torch.empty_like(kvsrc)
            qp, kp = qsrc.data_ptr(), kvsrc.data_ptr() + ctx.kv_col * es
            vp = kp + hd * es
            dqp, dkp = dq.data_ptr(), dkv.data_ptr() + ctx.kv_col * es
            dvp = dkp + hd * es
            if f32:
                qpl = _planes_like(dq)
                kvpl = (ctx.shared.get_planes(dkv) if ctx.shared is not None else _planes_like(dkv))
                if qpl is not None and kvpl is not None:
                    _pl.attach(dq, qpl)
                    if ctx.shared is None:
                        _pl.attach(dkv, kvpl)
                    pq, q_ps = qpl.data_ptr(), qpl.stride(0)
                    pk, kv_ps = kvpl.data_ptr() + ctx.kv_col * 2, kvpl.stride(0)
                    pv = pk + hd * 2
        else:
            dqkv = torch.empty_like(qsrc)
            qp = qsrc.data_ptr()
            kp, vp = qp + hd * es, qp + 2 * hd * es
            dqp = dqkv.data_ptr()
            dkp, dvp = dqp + hd * es, dqp + 2 * hd * es
            if f32:
                pl = _planes_like(dqkv)
                if pl is not None:
                    _pl.attach(dqkv, pl)
                    pq, q_ps = pl.data_ptr(), pl.stride(0)
                    pk, pv, kv_ps = pq + hd * 2, pq + 2 * hd * 2, q_ps
        if f32:
            _pl.f32(do)  # the kernels read dO's fp32 values
            # dQ/dK/dV feed only the projections' dgrad / wgrad GEMMs (their planes): planes only
            only = bool(pq) and _pl.grad_planes_ok(qsrc) and (not ctx.cross or ctx.shared is not None
                                                               or _pl.grad_planes_ok(kvsrc))
            C.attn_f32_bwd(qp, kp, vp, qs, ks, vs, o.data_ptr(), do.data_ptr(), os_, lse.data_ptr(), delta.data_ptr(),
                           dqp, dkp, dvp, _native.ptr(ctx.kpad), B, H, Sq, Sk, ctx.mode, _LOG2E / math.sqrt(hd),
                           1.0 / math.sqrt(hd), pq, pk, pv, q_ps, kv_ps, int(only), _native.stream())
            if only:
                if ctx.cross:
                    dq._smi_planes_only = True
                    if ctx.shared is not None:
                        ctx.shared.planes_only = True
                    else:
                        dkv._smi_planes_only = True
                else:
                    dqkv._smi_planes_only = True
        else:
            C.attn_bwd(qp, kp, vp, qs, ks, vs, o.data_ptr(), do.data_ptr(), os_, lse.data_ptr(), delta.data_ptr(), dqp,
                       dkp, dvp, _native.ptr(ctx.kpad), B, H, Sq, Sk, ctx.mode, _LOG2E / math.sqrt(hd),
                       1.0 / math.sqrt(hd), _native.stream())
        if ctx.cross:
            # a shared kv gradient is read by its producer (ops.linear.ConcatLinearFn)
            return dq, (None if ctx.shared is not None else dkv), None, None, None, None, None, None
        return dqkv, None, None, None, None, None, None, None


def self_attention(qkv, num_heads, mode="none", key_padding=None):
    """qkv [B,S,H*3*hd] (per-head interleaved) -> [B,S,H*hd]."""
    return _AttnCore.apply(qkv, None, num_heads, MODES[mode] if not isinstance(mode, int) else mode, key_padding,
                           False, 0, None)


def cross_attention(q, kv, num_heads, mode="none", key_padding=None, kv_col=0, shared=None):
    """q [B,Sq,H*hd], kv [B,Sk,H*2*hd] (per-head [k|v]) -> [B,Sq,H*hd].  GPU: ``kv`` may be a wider
    concatenated projection [B,Sk,W] read from column ``kv_col``; with ``shared`` (a SharedGrad)
    the kv gradient is written into ``shared``'s buffer at the same columns."""
    return _AttnCore.apply(q, kv, num_heads, MODES[mode] if not isinstance(mode, int) else mode, key_padding, True,
                           int(kv_col), shared)
