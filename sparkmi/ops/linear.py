"""Linear layer and fused FFN with MFMA GEMMs, fused epilogues and direct fp32 weight-grad
accumulation.

y = dropout_p(act(x @ W^T + b)).  Reference call sites: every nn.Linear of transformer.py
(qkv_layer :71, linear_layer :72, kv_layer/q_layer :175-176, FFN :107-117, vocab projection
:271), the MLP (distributed_multilayer_perceptron.py:47-53) and the CNN classifier
(distributed_cnn.py:74-78).

GPU paths, chosen by the activation dtype:
  * fp32 (reference precision): csrc/kernels/gemm_sp*.hip — every operand as three exact bf16
    planes (sparkmi/ops/planes.py: weights split by the optimizer, activations split once where
    produced and shared by the forward and weight-gradient GEMMs), six bf16 products per fp32
    product on v_mfma_f32_32x32x16_bf16, the same fused epilogues; shapes outside its tiling run
    csrc/kernels/gemm_f32.hip on the fp32 operands;
  * bf16 (bf16 weight shadow, fp32 master/grad): csrc/kernels/gemm.hip (16x16x32 bf16 MFMA)
    whenever the shape fits (K % 64 == 0, rows 16-B aligned), the fp32 kernel on upcast
    operands otherwise (no vendor-library GEMM anywhere).
  * forward: ONE kernel = GEMM + bias + ReLU + dropout epilogue (counter-based mask, nothing
    saved but the output);
  * backward: dgrad GEMM (bf16 out), wgrad GEMM accumulating fp32 straight into the flat
    gradient buffer (split-K atomics), bias grad by a HIP column-sum kernel.
``ffn()`` fuses PositionwiseFeedForward (Linear -> ReLU -> Dropout -> Linear): its backward
applies the ReLU/dropout mask inside linear2's dgrad epilogue (no elementwise pass).
CPU path: fp32 torch math with the identical dropout mask.
"""
import torch

from .. import _native
from . import gemm as G
from . import planes as _pl
from . import rng as _rng
from . import _grad
from ._grad import bf16_weight, grad_buf, grad_ready

ACTS = {None: 0, "none": 0, "relu": 1, "sigmoid": 2}


_GROUP_LIMIT = 1 << 31  # descriptor / 32-bit offset range of the grouped wgrad launches


def _groupable(*ts):
    return all(t.numel() * t.element_size() < _GROUP_LIMIT for t in ts)


def _r4(n):
    return (n + 3) // 4 * 4


def _pad2(t, rows, cols):
    """Zero-padded copy of a 2-D tensor (or the tensor itself when already that shape)."""
    if t is None or tuple(t.shape) == (rows, cols):
        return t
    out = t.new_zeros(rows, cols)
    out[:t.shape[0], :t.shape[1]] = t
    return out


# FFN hidden activation as planes + positivity mask (no fp32 tensor; -400 MB of activations per
# step, round 3c); False keeps fp32
_FFN_MASK = True


def _fwd32_any(x2, w, bias, act, rng, salt, p):
    """fp32 forward for any shape: the kernel needs K % 4 (float4 k-loads); a ragged K is
    zero-padded (zeros add nothing).  Ragged N is handled by the kernel's scalar epilogue."""
    M, K = x2.shape
    N = w.shape[0]
    if not G.supported32(M, N, K, x2, w, mode=0):
        x2, w = _pad2(x2.contiguous(), M, _r4(K)), _pad2(w.contiguous(), N, _r4(K))
    return G.fwd32(x2, w, bias, act, rng, salt, _rng.threshold(p), _rng.scale(p))


def _dgrad32_any(g2, w, resid=None, dact_y=None, dscale=1.0):
    """fp32 dgrad for any shape: the reduction dim N (dy's columns, W's rows) and the output
    dim K need multiples of 4 for the kernel's float4 loads; ragged ones are zero-padded."""
    M, N = g2.shape
    K = w.shape[1]
    if G.supported32(M, K, N, g2, w, resid, dact_y, mode=1):
        return G.dgrad32(g2, w, resid=resid, dact_y=dact_y, dscale=dscale)
    N4, K4 = _r4(N), _r4(K)
    dx = G.dgrad32(_pad2(g2.contiguous(), M, N4), _pad2(w.contiguous(), N4, K4),
                   resid=_pad2(resid.contiguous(), M, K4) if resid is not None else None,
                   dact_y=_pad2(dact_y.contiguous(), M, K4) if dact_y is not None else None, dscale=dscale)
    return dx[:, :K] if K4 != K else dx


def _wgrad32_any(gw, dy2, x2, gb=None):
    """gw[N,K] (+)= dy^T x, gb += colsum(dy), fp32, any shape (ragged dims zero-padded into a
    temporary that is then added)."""
    N, K = gw.shape
    M = dy2.shape[0]
    if G.supported32(N, K, M, dy2, x2, mode=2) and gw.is_contiguous():
        G.wgrad32(dy2, x2, gw, gb=gb)
        return
    M4, N4, K4 = _r4(M), _r4(N), _r4(K)
    t = torch.zeros(N4, K4, device=gw.device, dtype=torch.float32)
    tb = torch.zeros(N4, device=gw.device, dtype=torch.float32) if gb is not None else None
    G.wgrad32(_pad2(dy2.contiguous(), M4, N4), _pad2(x2.contiguous(), M4, K4), t, gb=tb)
    gw.add_(t[:N, :K])
    if gb is not None:
        gb.add_(tb[:N])


def _wgrad_accumulate(gw: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor, gb=None, ready=None):
    """gw (fp32 [N,K]) += dy2^T @ x2 with fp32 accumulation on the GPU; gb (fp32 [N], optional)
    += column sums of dy2 — fused into sparkmi's wgrad kernel, a column-sum kernel otherwise.
    Returns True when the split-K fold was deferred (then ``ready`` is reported final by the
    end-of-backward flush, sparkmi/ops/_grad.py); otherwise the caller reports it."""
    N, K = gw.shape
    M = dy2.shape[0]
    if dy2.dtype == torch.float32 and G.SP and gw.is_contiguous() and N % 8 == 0 and K % 8 == 0 and (
            gb is None or gb.is_contiguous()):
        dyp, xp = _pl.cached(dy2), _pl.cached(x2)
        if dyp is not None and xp is not None:
            if ready is not None and _grad.WGRAD_GROUP and _groupable(dyp, xp):
                _grad.defer_wgrad_group(dyp, xp, gw, gb, ready, _native.stream())
                return True
            if G.sp_wgrad(dyp, xp, gw, gb):
                return False
    if dy2.dtype == torch.float32:
        _pl.f32(dy2)  # a planes-only gradient / activation on a path that reads fp32
        _pl.f32(x2)
        if (ready is not None and _grad.WGRAD_GROUP and G.supported32(N, K, M, dy2, x2, mode=2)
                and gw.is_contiguous() and _groupable(dy2, x2) and (gb is None or gb.is_contiguous())):
            _grad.defer_wgrad_group(dy2, x2, gw, gb, ready, _native.stream())
            return True
        _wgrad32_any(gw, dy2, x2, gb)
        return False
    if (ready is not None and _grad.WGRAD_GROUP and G.supported(N, K, M, dy2, x2, mode=2) and gw.is_contiguous()
            and (gb is None or gb.is_contiguous()) and dy2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16
            and _groupable(dy2, x2)):
        _grad.defer_wgrad_group(dy2, x2, gw, gb, ready, _native.stream())
        return True
    if G.supported(N, K, M, dy2, x2, mode=2) and gw.is_contiguous():
        return G.wgrad(dy2, x2, gw, gb=gb, ready=ready) is True
    # shapes outside the bf16 kernel's tiling: the fp32 kernel on upcast operands
    _wgrad32_any(gw, dy2.float(), x2.float(), gb)
    return False


def _dgrad(g2, w_bf, resid=None, dact_y=None, dscale=1.0, wp=None, out_planes=False, need_f32=True, dmask=None):
    """dX = dY W (+resid) (x relu'/dropout mask); fp32: on the split-plane GEMM from dY's planes.
    ``need_f32=False`` with ``out_planes``: dX as planes only (a placeholder fp32 tensor).
    ``dmask``: the positivity mask written by the producing forward epilogue, used instead of
    ``dact_y`` when that is a planes-only placeholder (filled here if a fallback needs it)."""
    M, N = g2.shape
    K = w_bf.shape[1]
    if g2.dtype == torch.float32:
        if wp is not None and G.SP and G._sp_ok(g2):
            r = G.sp_dgrad(_pl.of(g2, kpad=N % 32 != 0), wp, M, K, N, resid=resid,
                           dact_y=dact_y if dmask is None else None, dscale=dscale, out_planes=out_planes,
                           need_f32=need_f32 or not out_planes, dmask=dmask)
            if r is not None:
                dx, dxp = r
                if dx is None:
                    return _pl.placeholder((M, K), dxp, g2.device)
                if dxp is not None:
                    _pl.attach(dx, dxp)
                return dx
        return _dgrad32_any(_pl.f32(g2), w_bf, resid, _pl.f32(dact_y) if dact_y is not None else None, dscale)
    if G.supported(M, K, N, g2, w_bf, resid, dact_y, mode=1):
        return G.dgrad(g2, w_bf, resid=resid, dact_y=dact_y, dscale=dscale)
    f32 = [t.float() if t is not None else None for t in (g2, w_bf, resid, dact_y)]
    return _dgrad32_any(*f32[:2], f32[2], f32[3], dscale).to(g2.dtype)


def compute_weight(p: torch.Tensor, dtype) -> torch.Tensor:
    """The weight operand for activations of ``dtype``: the fp32 master itself, or its bf16 shadow."""
    return p.detach() if dtype == torch.float32 else bf16_weight(p)


def _fwd_sp(x2, wp, N, bias, act, p, rng, salt, out_planes=False, relu_mask=None):
    """fp32 forward on the split-plane GEMM (x2's planes: cached or split now); None if not covered."""
    M, K = x2.shape
    if wp is None or not G.SP or not G._sp_ok(x2) or act not in (0, 1):
        return None
    if relu_mask is not None:  # planes + positivity mask, no fp32 tensor (FFNFn)
        r = G.sp_fwd(_pl.of(x2), wp, M, N, K, bias, act, rng, salt, _rng.threshold(p), _rng.scale(p),
                     out_planes=True, mask=relu_mask)
        if r is not None:
            return _pl.placeholder((M, N), r[1], x2.device)
    r = G.sp_fwd(_pl.of(x2), wp, M, N, K, bias, act, rng, salt, _rng.threshold(p), _rng.scale(p),
                 out_planes=out_planes)
    if r is None:
        return None
    y, yp = r
    if yp is not None:
        _pl.attach(y, yp)
    return y


def _wplanes(weight):
    return _pl.weight(weight) if G.SP and weight.dim() == 2 and weight.shape[1] % 8 == 0 else None


def _fwd_native(x2, weight, bias, act, p, rng, salt, w_bf=None, out_planes=False, wp=None, relu_mask=None):
    N, K = weight.shape
    M = x2.shape[0]
    if x2.dtype == torch.float32:
        y = _fwd_sp(x2, wp if wp is not None else _wplanes(weight), N, bias, act, p, rng, salt, out_planes,
                    relu_mask)
        if y is not None:
            return y
        return _fwd32_any(_pl.f32(x2), weight.detach(), bias, act, rng, salt, p)
    w = w_bf if w_bf is not None else bf16_weight(weight)
    if G.supported(M, N, K, x2, w, mode=0) and act in (0, 1):
        return G.fwd(x2, w, bias, act, rng, salt, _rng.threshold(p), _rng.scale(p))
    # shapes outside the bf16 kernel's tiling (or sigmoid): the fp32 kernel on upcast operands
    return _fwd32_any(x2.float(), weight.detach(), bias, act, rng, salt, p).to(x2.dtype)


def _ref_fwd(x2, weight, bias, act, p, seed, salt):
    y2 = x2.float() @ weight.float().t()
    if bias is not None:
        y2 = y2 + bias.float()
    if act == 1:
        y2 = torch.relu(y2)
    elif act == 2:
        y2 = torch.sigmoid(y2)
    if p > 0:
        y2 = y2 * _rng.keep_mask(y2.shape, p, seed, salt, y2.device).to(y2.dtype) * _rng.scale(p)
    return y2


def _ref_act_bwd(g2, y2, act, p, seed, salt):
    if act == 1:
        return g2 * (y2.float() > 0).to(g2.dtype) * (_rng.scale(p) if p > 0 else 1.0)
    if act == 2:
        s = y2.float()
        g2 = g2 * s * (1 - s)
    if p > 0:
        g2 = g2 * _rng.keep_mask(g2.shape, p, seed, salt, g2.device).to(g2.dtype) * _rng.scale(p)
    return g2


class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, act, p, rng, salt, x_slot=None, planes=0):
        shp = x.shape
        K = shp[-1]
        N = weight.shape[0]
        x2 = x.reshape(-1, K)
        ctx.act, ctx.p, ctx.rng, ctx.salt = act, p, rng, salt
        ctx.native = _native.use_native(x)
        if ctx.native:
            x2 = x2.contiguous()
            y2 = _fwd_native(x2, weight, bias, act, p, rng, salt, out_planes=bool(planes & 1))
            ctx.x_planes = _pl.cached(x2)  # kept for the weight-gradient GEMM
            ctx.seed = 0
        else:
            ctx.seed = rng.current() if p > 0 else 0
            y2 = _ref_fwd(x2, weight, bias, act, p, ctx.seed, salt).to(x.dtype)
        ctx.x_slot, ctx.dx_planes = x_slot, bool(planes & 2)
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
            if act or p > 0 or not dy2.is_contiguous():
                _pl.f32(dy2)  # read as fp32 below
            dy2 = dy2.contiguous()
            if act or p > 0:
                g2 = torch.empty_like(dy2)
                fn = C.act_drop_bwd_f32 if dy2.dtype == torch.float32 else C.act_drop_bwd
                fn(dy2.data_ptr(), _native.ptr(y2), g2.data_ptr(), dy2.numel(), act, ctx.rng.ptr(),
                   ctx.salt, _rng.threshold(p), _rng.scale(p), _native.stream())
            else:
                g2 = dy2
            resid = _slot_grad(ctx.x_slot, g2.shape[0])
            f32 = g2.dtype == torch.float32
            wp = _wplanes(weight) if f32 else None
            dx = _dgrad(g2, compute_weight(weight, g2.dtype), resid=resid, wp=wp,
                        out_planes=ctx.dx_planes) if ctx.needs_input_grad[0] else None
            bgrad = grad_buf(bias) if bias is not None else None
            if f32 and G.SP and ctx.x_planes is not None:
                _pl.attach(x2, ctx.x_planes)
                _pl.of(g2, kpad=g2.shape[1] % 32 != 0)
            with _grad.side(g2.device, g2, x2):
                deferred = _wgrad_accumulate(gw, g2, x2, bgrad, ready=(weight, bias))
        else:
            g2 = _ref_act_bwd(dy2.float(), y2, act, p, ctx.seed, ctx.salt)
            resid = _slot_grad(ctx.x_slot, g2.shape[0])
            dx = None
            if ctx.needs_input_grad[0]:
                dx = g2 @ weight.float()
                if resid is not None:
                    dx = dx + resid.float()
                dx = dx.to(dy.dtype)
            gw.add_(g2.t() @ x2.float())
            if bias is not None:
                grad_buf(bias).add_(g2.sum(0))
            deferred = False
        if not deferred:
            grad_ready(weight, bias)
        if dx is not None:
            dx = dx.reshape(*dy.shape[:-1], K)
        return dx, None, None, None, None, None, None, None, None


def _slot_grad(slot, rows):
    """The residual gradient parked for this op's input (see _grad.ResidualGrad), 2-D, or None."""
    if slot is None:
        return None
    g = slot.take()
    return g.reshape(rows, -1).contiguous() if g is not None else None


def linear(x, weight, bias=None, act=None, p=0.0, rng=None, salt=0, x_slot=None, out_planes=False, dx_planes=False):
    """y = dropout_p(act(x @ weight^T + bias)); act in {None, 'relu', 'sigmoid'}.  ``x_slot``:
    a ResidualGrad whose parked gradient is added to dX in the dgrad epilogue.  fp32 GPU path:
    ``out_planes`` / ``dx_planes`` make the forward / dgrad epilogue also write the split planes of
    y / dX (sparkmi/ops/planes.py) for a consumer that reads planes (the attention kernels)."""
    a = ACTS[act] if not isinstance(act, int) else act
    if a == 2 and p > 0:
        raise ValueError("sigmoid + dropout epilogue is not supported")
    if rng is None:
        from .layernorm import _NULL_RNG
        rng, p = _NULL_RNG, 0.0
    return LinearFn.apply(x, weight, bias, a, float(p), rng, int(salt), x_slot,
                          (1 if out_planes else 0) | (2 if dx_planes else 0))


class FFNFn(torch.autograd.Function):
    """y = linear2(dropout(relu(linear1(x)))) with a single saved hidden activation."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, p, rng, salt, x_slot=None):
        shp = x.shape
        D = shp[-1]
        x2 = x.reshape(-1, D)
        ctx.p, ctx.rng, ctx.salt = p, rng, salt
        ctx.native = _native.use_native(x)
        if ctx.native:
            x2 = x2.contiguous()
            # the hidden activation feeds linear2's GEMMs (planes) and linear2's dgrad epilogue (only
            # its sign): planes + a 4-bit-per-4-columns positivity mask, no fp32 tensor
            H = w1.shape[0]
            mask = (torch.empty(x2.shape[0], (H + 3) // 4, device=x2.device, dtype=torch.uint8)
                    if _pl.PLANES_ONLY and _FFN_MASK and x2.dtype == torch.float32 and G.SP else None)
            h = _fwd_native(x2, w1, b1, 1, p, rng, salt, out_planes=True, relu_mask=mask)
            ctx.h_mask = mask if (mask is not None and _pl.planes_only(h)) else None
            y = _fwd_native(h, w2, b2, 0, 0.0, rng, 0)
            ctx.x_planes, ctx.h_planes = _pl.cached(x2), _pl.cached(h)
            ctx.seed = 0
        else:
            ctx.seed = rng.current() if p > 0 else 0
            h = _ref_fwd(x2, w1, b1, 1, p, ctx.seed, salt).to(x.dtype)
            y = _ref_fwd(h, w2, b2, 0, 0.0, 0, 0).to(x.dtype)
        ctx.x_slot = x_slot
        ctx.save_for_backward(x2, h, w1, b1, w2, b2)
        return y.reshape(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, h, w1, b1, w2, b2 = ctx.saved_tensors
        D = w2.shape[0]
        dy2 = dy.reshape(-1, D)
        p = ctx.p
        if ctx.native:
            dy2 = dy2.contiguous()
            f32 = dy2.dtype == torch.float32
            if f32 and G.SP:
                if ctx.x_planes is not None:
                    _pl.attach(x2, ctx.x_planes)
                if ctx.h_planes is not None:
                    _pl.attach(h, ctx.h_planes)
            # dh_pre = (dy @ W2) * relu'/dropout mask (from the saved output h), fused epilogue
            # (fp32: its planes written by the same epilogue, for linear1's dgrad and wgrad)
            if not dy2.is_contiguous():
                _pl.f32(dy2)
            # dh feeds only linear1's dgrad / wgrad, both on its planes: planes only
            dh = _dgrad(dy2, compute_weight(w2, dy2.dtype), dact_y=h, dscale=_rng.scale(p),
                        wp=_wplanes(w2) if f32 else None, out_planes=True, need_f32=not _pl.PLANES_ONLY,
                        dmask=getattr(ctx, "h_mask", None))
            gw2, gb2, gw1, gb1 = grad_buf(w2), grad_buf(b2), grad_buf(w1), grad_buf(b1)
            with _grad.side(dy2.device, dy2, h):
                if not _wgrad_accumulate(gw2, dy2, h, gb2, ready=(w2, b2)):
                    grad_ready(w2, b2)
            resid = _slot_grad(ctx.x_slot, dh.shape[0])
            dx = _dgrad(dh, compute_weight(w1, dh.dtype), resid=resid,
                        wp=_wplanes(w1) if f32 else None) if ctx.needs_input_grad[0] else None
            with _grad.side(dh.device, dh, x2):
                if not _wgrad_accumulate(gw1, dh, x2, gb1, ready=(w1, b1)):
                    grad_ready(w1, b1)
        else:
            g = dy2.float()
            grad_buf(w2).add_(g.t() @ h.float())
            grad_buf(b2).add_(g.sum(0))
            grad_ready(w2, b2)
            dh = _ref_act_bwd(g @ w2.float(), h, 1, p, ctx.seed, ctx.salt)
            resid = _slot_grad(ctx.x_slot, dh.shape[0])
            dx = None
            if ctx.needs_input_grad[0]:
                dx = dh @ w1.float()
                if resid is not None:
                    dx = dx + resid.float()
                dx = dx.to(dy.dtype)
            grad_buf(w1).add_(dh.t() @ x2.float())
            grad_buf(b1).add_(dh.sum(0))
            grad_ready(w1, b1)
        if dx is not None:
            dx = dx.reshape(dy.shape)
        return dx, None, None, None, None, None, None, None, None


# ConcatLinearFn.backward: launch the projection's dgrad before forking the queued weight-gradient
# group onto the side stream (True) or after it (False, rounds 3-5)
CONCAT_DGRAD_FIRST = True


class ConcatLinearFn(torch.autograd.Function):
    """y = x @ W^T + b over linears stored back to back in the flat buffer (FlatParams.concat):
    one GEMM in place of several on the same input.  The consumers read column slices of y and
    write their gradients into ``shared`` (a SharedGrad) instead of returning them, so the
    backward is ONE dgrad GEMM with K = the summed widths (the sum over consumers happens in the
    MFMA accumulators, no elementwise adds) and ONE weight-gradient GEMM."""

    @staticmethod
    def forward(ctx, x, wviews, bviews, shape, params, shared):
        ctx.set_materialize_grads(False)
        N, K = shape
        wm, wg, ws = wviews[:3]
        bm, bg = bviews[0], bviews[1]
        x2 = x.reshape(-1, K).contiguous()
        w = wm.view(N, K)
        wp = wviews[3] if len(wviews) > 3 and x2.dtype == torch.float32 and G.SP else None
        y2 = _fwd_native(x2, w, bm, 0, 0.0, None, 0, w_bf=ws.view(N, K) if ws is not None else None, wp=wp)
        ctx.wviews, ctx.bg, ctx.shape, ctx.params, ctx.shared = wviews, bg, shape, params, shared
        ctx.x_planes, ctx.wp = _pl.cached(x2), wp
        ctx.save_for_backward(x2)
        return y2.reshape(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, _unused):
        (x2,) = ctx.saved_tensors
        N, K = ctx.shape
        wm, wg, ws = ctx.wviews[:3]
        g = ctx.shared.take()
        if g is None:  # no consumer produced a gradient
            grad_ready(*ctx.params)
            return None, None, None, None, None, None
        # every consumer of this projection (the decoder) has finished its backward: its queued
        # weight gradients run on a side stream beside the rest (the encoder's backward).  The
        # fork goes AFTER this projection's dgrad (CONCAT_DGRAD_FIRST): the side stream waits for
        # it, so the group's one-workgroup-per-CU tiles do not take the chip from the dgrad the
        # whole encoder backward waits on
        if not CONCAT_DGRAD_FIRST:
            _grad.flush_groups_async(g.device)
        g2 = g.reshape(-1, N)
        w = wm.view(N, K) if g2.dtype == torch.float32 else ws.view(N, K)
        dx = _dgrad(g2, w, wp=ctx.wp) if ctx.needs_input_grad[0] else None
        if CONCAT_DGRAD_FIRST:
            _grad.flush_groups_async(g.device)
        if ctx.wp is not None and ctx.x_planes is not None:
            _pl.attach(x2, ctx.x_planes)
            _pl.of(g2, kpad=N % 32 != 0)
        with _grad.side(g2.device, g2, x2):
            if not _wgrad_accumulate(wg.view(N, K), g2, x2, ctx.bg, ready=ctx.params):
                grad_ready(*ctx.params)
        if dx is not None:
            dx = dx.reshape(*g.shape[:-1], K)
        return dx, None, None, None, None, None


def concat_linear(x, flat, linears, shared):
    """One GEMM for several nn.Linear on the same input whose weights (and biases) FlatParams
    stored back to back; returns y [.., sum N_i] or None when the layout does not allow it.
    Consumers must route their gradient through ``shared`` (see ConcatLinearFn)."""
    ws = [l.weight for l in linears]
    bs = [l.bias for l in linears]
    if any(b is None for b in bs) or len({tuple(w.shape[1:]) for w in ws}) != 1:
        return None
    wv, bv = flat.concat(ws), flat.concat(bs)
    if wv is None or bv is None or (x.dtype == torch.bfloat16 and wv[2] is None):
        return None
    if x.dtype == torch.float32 and x.is_cuda and G.SP:
        wv = tuple(wv) + (flat.concat_planes(ws),)
    N, K = sum(w.shape[0] for w in ws), ws[0].shape[1]
    params = tuple(p for pair in zip(ws, bs) for p in pair)
    return ConcatLinearFn.apply(x, wv, bv, (N, K), params, shared)


def ffn(x, linear1, linear2, p=0.0, rng=None, salt=0, x_slot=None):
    if rng is None:
        from .layernorm import _NULL_RNG
        rng, p = _NULL_RNG, 0.0
    return FFNFn.apply(x, linear1.weight, linear1.bias, linear2.weight, linear2.bias, float(p), rng, int(salt),
                       x_slot)
