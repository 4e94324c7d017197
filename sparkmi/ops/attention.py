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
GPU: csrc/kernels/attention.hip (flash-style fwd; dQ and dK/dV backward kernels, no S x S
tensor in HBM).  CPU: torch reference math in fp32.
"""
import math

import torch

from .. import _native

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


class _AttnCore(torch.autograd.Function):
    """Shared autograd core.  ``views`` describe (base tensor, offset, (sb, ss, sh)) for q/k/v."""

    @staticmethod
    def forward(ctx, qsrc, kvsrc, H, mode, key_padding, cross):
        ctx.H, ctx.mode, ctx.cross = H, mode, cross
        ctx.native = _native.use_native(qsrc)
        if not ctx.native:
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
        B, Sq = qsrc.shape[0], qsrc.shape[1]
        if cross:
            kvsrc = kvsrc.contiguous()
            hd = qsrc.shape[2] // H
            Sk = kvsrc.shape[1]
            qp, qs = qsrc.data_ptr(), (Sq * H * hd, H * hd, hd)
            kp, ks = kvsrc.data_ptr(), (Sk * 2 * H * hd, 2 * H * hd, 2 * hd)
            vp, vs = kp + hd * 2, ks
        else:
            hd = qsrc.shape[2] // (3 * H)
            Sk = Sq
            qp, qs = qsrc.data_ptr(), (Sq * 3 * H * hd, 3 * H * hd, 3 * hd)
            kp, ks = qp + hd * 2, qs
            vp, vs = qp + 2 * hd * 2, qs
        if hd != 64:
            raise NotImplementedError("sparkmi attention kernel supports head_dim 64")
        o = torch.empty(B, Sq, H * hd, device=qsrc.device, dtype=torch.bfloat16)
        lse = torch.empty(B, H, Sq, device=qsrc.device, dtype=torch.float32)
        os_ = (Sq * H * hd, H * hd, hd)
        kpad = key_padding.to(torch.uint8).contiguous() if key_padding is not None else None
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
                return dqs.to(do.dtype), dkv.to(do.dtype), None, None, None, None
            dqkv = torch.cat([dq, dk, dv], dim=-1).permute(0, 2, 1, 3).reshape(B, S, -1)
            return dqkv.to(do.dtype), None, None, None, None, None
        C = _native.C()
        qsrc, kvsrc, o, lse = ctx.saved_tensors
        B, Sq, Sk, hd, qs, ks, vs, os_ = ctx.geom
        H = ctx.H
        do = do.contiguous()
        delta = torch.empty(B, H, Sq, device=do.device, dtype=torch.float32)
        if ctx.cross:
            dq = torch.empty_like(qsrc)
            dkv = torch.empty_like(kvsrc)
            qp, kp = qsrc.data_ptr(), kvsrc.data_ptr()
            vp = kp + hd * 2
            dqp, dkp = dq.data_ptr(), dkv.data_ptr()
            dvp = dkp + hd * 2
        else:
            dqkv = torch.empty_like(qsrc)
            qp = qsrc.data_ptr()
            kp, vp = qp + hd * 2, qp + 4 * hd
            dqp = dqkv.data_ptr()
            dkp, dvp = dqp + hd * 2, dqp + 4 * hd
        C.attn_bwd(qp, kp, vp, qs, ks, vs, o.data_ptr(), do.data_ptr(), os_, lse.data_ptr(), delta.data_ptr(), dqp,
                   dkp, dvp, _native.ptr(ctx.kpad), B, H, Sq, Sk, ctx.mode, _LOG2E / math.sqrt(hd),
                   1.0 / math.sqrt(hd), _native.stream())
        if ctx.cross:
            return dq, dkv, None, None, None, None
        return dqkv, None, None, None, None, None


def self_attention(qkv, num_heads, mode="none", key_padding=None):
    """qkv [B,S,H*3*hd] (per-head interleaved) -> [B,S,H*hd]."""
    return _AttnCore.apply(qkv, None, num_heads, MODES[mode] if not isinstance(mode, int) else mode, key_padding,
                           False)


def cross_attention(q, kv, num_heads, mode="none", key_padding=None):
    """q [B,Sq,H*hd], kv [B,Sk,H*2*hd] (per-head [k|v]) -> [B,Sq,H*hd]."""
    return _AttnCore.apply(q, kv, num_heads, MODES[mode] if not isinstance(mode, int) else mode, key_padding, True)
