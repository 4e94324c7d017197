"""Linear layer with fused bias / activation / dropout epilogue and direct fp32 weight-grad
accumulation.

y = dropout_p(act(x @ W^T + b)).  Reference call sites: every nn.Linear of transformer.py
(qkv_layer :71, linear_layer :72, kv_layer/q_layer :175-176, FFN :107-117, vocab projection
:271), the MLP (distributed_multilayer_perceptron.py:47-53) and the CNN classifier
(distributed_cnn.py:74-78).

GPU path (bf16 activations, bf16 weight shadow, fp32 master/grad):
  * forward GEMM on MFMA: sparkmi's own HIP GEMM (csrc/kernels/gemm.hip) when the shape is
    supported, hipBLASLt (through torch.addmm) otherwise; the act+dropout epilogue is a HIP
    kernel (csrc/kernels/elementwise.hip) keyed by a counter-based mask (no mask tensor saved).
  * backward: dgrad GEMM, wgrad GEMM accumulated in fp32 into the flat gradient buffer
    (addmm with out_dtype=fp32, beta=1), bias grad by a HIP column-sum kernel.
CPU path: fp32 torch math with the identical dropout mask.
"""
import torch

from .. import _native
from . import rng as _rng
from ._grad import bf16_weight, grad_buf, grad_ready

ACTS = {None: 0, "none": 0, "relu": 1, "sigmoid": 2}

_colsum_part = {}


def _wgrad_accumulate(gw: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor):
    """gw (fp32 [N,K]) += dy2^T @ x2 with fp32 accumulation on the GPU."""
    try:
        torch.addmm(gw, dy2.t(), x2, out_dtype=torch.float32, out=gw)
        return
    except (TypeError, RuntimeError):
        pass
    gw.add_(torch.mm(dy2.t(), x2).float())


def _colsum(dy2: torch.Tensor, out: torch.Tensor):
    M, N = dy2.shape
    C = _native.C()
    rpb = 256
    nparts = (M + rpb - 1) // rpb
    key = (dy2.device, nparts * N)
    part = _colsum_part.get(key)
    if part is None or torch.cuda.is_current_stream_capturing():
        part = torch.empty(nparts * N, device=dy2.device, dtype=torch.float32)
        if not torch.cuda.is_current_stream_capturing():
            _colsum_part[key] = part
    C.colsum_bf16(dy2.data_ptr(), M, N, part.data_ptr(), rpb, out.data_ptr(), 1, _native.stream())


class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, act, p, rng, salt):
        shp = x.shape
        K = shp[-1]
        N = weight.shape[0]
        x2 = x.reshape(-1, K)
        ctx.act, ctx.p, ctx.rng, ctx.salt = act, p, rng, salt
        ctx.has_bias = bias is not None
        ctx.native = _native.use_native(x)
        if ctx.native:
            C = _native.C()
            x2 = x2.contiguous()
            w = bf16_weight(weight)
            if bias is not None:
                y2 = torch.addmm(bf16_weight(bias), x2, w.t())
            else:
                y2 = torch.mm(x2, w.t())
            if act or p > 0:
                C.bias_act_drop_fwd(y2.data_ptr(), 0, y2.data_ptr(), y2.numel(), N, act, rng.ptr(), salt,
                                    _rng.threshold(p), _rng.scale(p), _native.stream())
            ctx.seed = 0
        else:
            w = weight
            y2 = x2.float() @ w.float().t()
            if bias is not None:
                y2 = y2 + bias.float()
            if act == 1:
                y2 = torch.relu(y2)
            elif act == 2:
                y2 = torch.sigmoid(y2)
            ctx.seed = rng.current() if p > 0 else 0
            if p > 0:
                y2 = y2 * _rng.keep_mask(y2.shape, p, ctx.seed, salt, y2.device).to(y2.dtype) * _rng.scale(p)
            y2 = y2.to(x.dtype)
        # relu/sigmoid backward needs the output; identity+dropout recomputes the mask
        ctx.save_for_backward(x2, weight, bias, y2 if act else None)
        return y2.reshape(*shp[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, weight, bias, y2 = ctx.saved_tensors
        N, K = weight.shape
        dy2 = dy.reshape(-1, N)
        act, p = ctx.act, ctx.p
        gw = grad_buf(weight)
        if ctx.native:
            C = _native.C()
            dy2 = dy2.contiguous()
            if act or p > 0:
                g2 = torch.empty_like(dy2)
                C.act_drop_bwd(dy2.data_ptr(), _native.ptr(y2), g2.data_ptr(), dy2.numel(), act, ctx.rng.ptr(),
                               ctx.salt, _rng.threshold(p), _rng.scale(p), _native.stream())
            else:
                g2 = dy2
            dx = torch.mm(g2, bf16_weight(weight)) if ctx.needs_input_grad[0] else None
            _wgrad_accumulate(gw, g2, x2)
            if bias is not None:
                _colsum(g2, grad_buf(bias))
        else:
            g2 = dy2.float()
            if act == 1:
                g2 = g2 * (y2.float() > 0).to(g2.dtype) * (_rng.scale(p) if p > 0 else 1.0)
            else:
                if act == 2:
                    s = y2.float()
                    g2 = g2 * s * (1 - s)
                if p > 0:
                    g2 = g2 * _rng.keep_mask(g2.shape, p, ctx.seed, ctx.salt, g2.device).to(g2.dtype) * _rng.scale(p)
            dx = (g2 @ weight.float()).to(dy.dtype) if ctx.needs_input_grad[0] else None
            gw.add_(g2.t() @ x2.float())
            if bias is not None:
                grad_buf(bias).add_(g2.sum(0))
        grad_ready(weight, bias)
        if dx is not None:
            dx = dx.reshape(*dy.shape[:-1], K)
        return dx, None, None, None, None, None, None


def linear(x, weight, bias=None, act=None, p=0.0, rng=None, salt=0):
    """y = dropout_p(act(x @ weight^T + bias)); act in {None, 'relu', 'sigmoid'}."""
    a = ACTS[act] if not isinstance(act, int) else act
    if a == 2 and p > 0:
        raise ValueError("sigmoid + dropout epilogue is not supported")
    if rng is None:
        from .layernorm import _NULL_RNG
        rng, p = _NULL_RNG, 0.0
    return LinearFn.apply(x, weight, bias, a, float(p), rng, int(salt))
