"""Fused dropout + residual + LayerNorm (post-LN transformer sublayer epilogue).

y = LayerNorm(dropout_p(h) + residual) * gamma + beta, biased variance, eps inside the sqrt —
the reference's LayerNormalization (transformer.py:86-101) applied as in EncoderLayer /
DecoderLayer (transformer.py:130-139, :209-224).  GPU: one HIP kernel forward
(csrc/kernels/layernorm.hip), one kernel + a column-sum kernel backward; gamma/beta gradients
go straight into the fp32 flat gradient buffer.  CPU: the same math in fp32 torch.
"""
import torch

from .. import _native
from . import rng as _rng
from . import _grad
from . import planes as _pl
from ._grad import grad_buf, grad_ready


def _planes_for(t, D, M):
    """bf16 hi/mid/lo planes [3, M, D] for an fp32 output the split-plane GEMM will consume
    (sparkmi/ops/planes.py), or None (bf16 path, planes disabled, or a width the GEMM pads)."""
    from . import gemm as G
    if t.dtype != torch.float32 or not G.SP or D % 32:
        return None
    return torch.empty(3, M, D, device=t.device, dtype=torch.bfloat16)



def _ref_forward(h, r, gamma, beta, p, seed, salt, eps):
    x = h.float()
    if p > 0:
        x = x * _rng.keep_mask(x.shape, p, seed, salt, x.device).to(x.dtype) * _rng.scale(p)
    if r is not None:
        x = x + r.float()
    mean = x.mean(-1, keepdim=True)
    var = ((x - mean) ** 2).mean(-1, keepdim=True)
    rstd = 1.0 / torch.sqrt(var + eps)
    y = (x - mean) * rstd * gamma.float() + beta.float()
    return y, x, mean.reshape(-1), rstd.reshape(-1)


class AddDropoutLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, r, gamma, beta, p, rng, salt, eps, r_slot=None):
        D = h.shape[-1]
        M = h.numel() // D
        ctx.p, ctx.rng, ctx.salt, ctx.D, ctx.M = p, rng, salt, D, M
        ctx.has_r = r is not None
        ctx.r_slot = r_slot
        ctx.h_gplanes = _pl.grad_planes_ok(h)  # dh may be handed back as planes only
        if _native.use_native(h):
            C = _native.C()
            h = h.contiguous()
            r = r.contiguous() if r is not None else None
            y = torch.empty_like(h)
            xs = torch.empty_like(h)
            mean = torch.empty(M, device=h.device, dtype=torch.float32)
            rstd = torch.empty(M, device=h.device, dtype=torch.float32)
            if r is not None and r.dtype != h.dtype:
                raise TypeError(f"layernorm: residual dtype {r.dtype} != input dtype {h.dtype}")
            args = (h.data_ptr(), _native.ptr(r), gamma.data_ptr(), beta.data_ptr(), y.data_ptr(), xs.data_ptr(),
                    mean.data_ptr(), rstd.data_ptr(), M, D, eps, rng.ptr(), salt, _rng.threshold(p), _rng.scale(p))
            if h.dtype == torch.float32:
                yp = _planes_for(y, D, M)  # the next Linear's operand, written beside y
                C.ln_fwd_f32(*args, _native.ptr(yp), yp.stride(0) if yp is not None else 0, _native.stream())
                if yp is not None:
                    _pl.attach(y, yp)
            else:
                C.ln_fwd(*args, _native.stream())
            ctx.native = True
        else:
            seed = rng.current()
            ctx.seed = seed
            y, xs, mean, rstd = _ref_forward(h, r, gamma, beta, p, seed, salt, eps)
            y = y.to(h.dtype)
            ctx.native = False
        ctx.save_for_backward(xs, mean, rstd, gamma, beta)
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, mean, rstd, gamma, beta = ctx.saved_tensors
        D, M, p = ctx.D, ctx.M, ctx.p
        gg, gb = grad_buf(gamma), grad_buf(beta)
        if ctx.native:
            C = _native.C()
            dy = dy.contiguous()
            dres = torch.empty_like(dy) if ctx.has_r else None
            dh = torch.empty_like(dy)
            vpl = (D + 511) // 512
            rows_per_block = 4 * (2 if vpl <= 2 else 1)  # ln_bwd_kernel<VPL, RPW>
            nb = (M + rows_per_block - 1) // rows_per_block
            part = torch.empty(2, nb, D, device=dy.device, dtype=torch.float32)
            args = (dy.data_ptr(), xs.data_ptr(), mean.data_ptr(), rstd.data_ptr(), gamma.data_ptr(),
                    _native.ptr(dres), dh.data_ptr(), 0, part[0].data_ptr(), part[1].data_ptr(), nb,
                    0, 0, 1, M, D, ctx.rng.ptr(), ctx.salt, _rng.threshold(p), _rng.scale(p))
            if dy.dtype == torch.float32:
                dhp = _planes_for(dh, D, M)  # dY operand of the sublayer's last Linear (dgrad + wgrad)
                only = dhp is not None and ctx.h_gplanes  # ... which reads nothing else: planes only
                if only:
                    args = args[:6] + (0,) + args[7:]
                C.ln_bwd_f32(*args, _native.ptr(dhp), dhp.stride(0) if dhp is not None else 0, _native.stream())
                if dhp is not None:
                    _pl.attach(dh, dhp)
                    dh._smi_planes_only = only
            else:
                C.ln_bwd(*args, _native.stream())
            if _grad.LN_DEFER:  # folded with every other LayerNorm's at the end of the backward
                _grad.defer_ln_fold(part[0], part[1], nb, D, gg, gb, (gamma, beta), _native.stream())
            else:
                # dgamma / dbeta are off the critical path: reduce the partial rows on the side stream
                with _grad.side(dy.device, part):
                    C.ln_bwd_reduce(part[0].data_ptr(), part[1].data_ptr(), nb, D, gg.data_ptr(), gb.data_ptr(), 1,
                                    _native.stream())
        else:
            x = xs.reshape(M, D).float()
            g = dy.reshape(M, D).float()
            xhat = (x - mean[:, None]) * rstd[:, None]
            gl = g * gamma.float()
            dx = rstd[:, None] * (gl - gl.mean(-1, keepdim=True) - xhat * (gl * xhat).mean(-1, keepdim=True))
            gg.add_((g * xhat).sum(0))
            gb.add_(g.sum(0))
            dres = dx.reshape(dy.shape).to(dy.dtype) if ctx.has_r else None
            dhh = dx
            if p > 0:
                dhh = dhh * _rng.keep_mask((M, D), p, ctx.seed, ctx.salt, dx.device).to(dx.dtype) * _rng.scale(p)
            dh = dhh.reshape(dy.shape).to(dy.dtype)
        if not (ctx.native and _grad.LN_DEFER):
            grad_ready(gamma, beta)
        if ctx.r_slot is not None and dres is not None:
            ctx.r_slot.grad = dres  # added by the sibling linear's dgrad epilogue instead
            dres = None
        return dh, dres, None, None, None, None, None, None, None


def add_dropout_layernorm(h, residual, gamma, beta, p=0.0, rng=None, salt=0, eps=1e-5, r_slot=None):
    """LayerNorm(dropout_p(h) + residual); with ``r_slot`` the residual's gradient is handed to
    the linear that consumes the same tensor (see ResidualGrad) instead of returned."""
    if rng is None:
        p = 0.0
        rng = _NULL_RNG
    return AddDropoutLayerNorm.apply(h, residual, gamma, beta, float(p), rng, int(salt), float(eps), r_slot)


class _NullRNG:
    def ptr(self):
        return 0

    def current(self):
        return 0


_NULL_RNG = _NullRNG()
