"""Fused embedding -> stacked LSTM -> per-step linear head (csrc/kernels/lstm.hip).

``lstm_classifier(ids, h0, c0, params, ...)`` returns ``(pred [B,T,C], h_n [L,B,H], c_n)`` —
exactly ``fc_out(lstm(embedding(ids), (h0, c0))[0])`` of the reference model
(distributed_lstm.py:110-135), including nn.LSTM's inter-layer dropout.  GPU: one persistent
workgroup per sequence for the forward, one for BPTT; each sequence's weight gradients go to a
slab that one kernel sums in sequence order into ``param.grad`` (flat fp32 buffers), and the
embedding-table gradient is a sorted segment sum — bit-reproducible, no float atomics; the
embedding rows equal to ``padding_idx`` get no gradient.  CPU: the identical math written with torch ops (same counter-hash dropout masks),
which is what the GPU kernel is tested against.
"""
import torch

from .. import _native
from . import rng as _rng
from ._grad import grad_buf, grad_ready


def unpack(params, L):
    emb = params[0]
    layers = [params[1 + 4 * i:5 + 4 * i] for i in range(L)]
    w_fc, b_fc = params[1 + 4 * L], params[2 + 4 * L]
    return emb, layers, w_fc, b_fc


def reference_forward(ids, h0, c0, params, L, p=0.0, step_seed=0, salt=0, padding_idx=None):
    """Torch reference (autograd-capable): embedding, L LSTM layers (gate order i,f,g,o), dropout
    between layers with the kernel's counter-hash mask, linear head at every step."""
    emb, layers, w_fc, b_fc = unpack(params, L)
    B, T = ids.shape
    H = layers[0][1].shape[1]
    x = torch.nn.functional.embedding(ids, emb, padding_idx=padding_idx)
    mask = None
    if p > 0:
        mask = _rng.keep_mask((B, T, L, H), p, step_seed, salt, ids.device)
    hs, cs = [], []
    for li, (w_ih, w_hh, b_ih, b_hh) in enumerate(layers):
        h = h0[li] if h0 is not None else x.new_zeros(B, H)
        c = c0[li] if c0 is not None else x.new_zeros(B, H)
        outs = []
        for t in range(T):
            z = x[:, t] @ w_ih.t() + b_ih + h @ w_hh.t() + b_hh
            i, f, g, o = z.chunk(4, dim=1)
            i, f, g, o = torch.sigmoid(i), torch.sigmoid(f), torch.tanh(g), torch.sigmoid(o)
            c = f * c + i * g
            h = o * torch.tanh(c)
            outs.append(h)
        hs.append(h)
        cs.append(c)
        x = torch.stack(outs, 1)
        if mask is not None and li + 1 < L:
            x = x * mask[:, :, li, :].to(x.dtype) * _rng.scale(p)
    pred = x @ w_fc.t() + b_fc
    return pred, torch.stack(hs), torch.stack(cs)


def supported(E, H, L, C):
    return _native.has_native() and bool(_native.C().lstm_supported(E, H, L, C))


class LSTMFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, h0, c0, meta, *params):
        return LSTMFn._forward(ctx, ids, h0, c0, meta, params, None)

    @staticmethod
    def _forward(ctx, ids, h0, c0, meta, params, labels):
        """The forward launch; ``labels``: also the fused last-step CE (returns its extra outputs)."""
        ctx.set_materialize_grads(False)  # unused outputs get no zero-filled gradients
        L, p, rng, salt, pad_idx = meta[:5]
        # the model's ticket block (meta[6]) or, for a bare op call, the per-device shared one
        tick = meta[6] if len(meta) > 6 and meta[6] is not None else _ce_ticket(ids.device)
        ctx.tick = tick
        emb, layers, w_fc, b_fc = unpack(params, L)
        B, T = ids.shape
        E, H, C = emb.shape[1], layers[0][1].shape[1], w_fc.shape[0]
        dev = ids.device
        ids = ids.to(torch.int64).contiguous()
        if not all(t.is_contiguous() and t.dtype == torch.float32 for t in params):
            raise ValueError("LSTM parameters must be contiguous fp32")
        # the fused-CE step returns (loss, pred[:, -1]) only: no [B, T, C] head output is computed
        pred = torch.empty(B, T, C, device=dev, dtype=torch.float32) if labels is None else None
        last = torch.empty(B, C, device=dev, dtype=torch.float32)  # pred[:, -1] written by the kernel too
        hn = torch.empty(L, B, H, device=dev, dtype=torch.float32)
        cn = torch.empty_like(hn)
        ws = torch.empty(B, L, T, 6 * H, device=dev, dtype=torch.float32)
        h0c = h0.float().contiguous() if h0 is not None else None
        c0c = c0.float().contiguous() if c0 is not None else None
        thresh = _rng.threshold(p)
        ce = None
        if labels is not None:
            labels = labels.to(torch.int64).contiguous()
            ce = (torch.empty(B, device=dev, dtype=torch.float32), torch.empty(B, C, device=dev, dtype=torch.float32),
                  torch.empty((), device=dev, dtype=torch.float32), tick)
        # the embedding backward's id ordering, made by this launch on CUs the recurrence leaves
        # idle (csrc/kernels/lstm.hip lstm_emb_side); the backward only sums
        plan_ws = None
        if (EMB_IN_FORWARD and ctx.needs_input_grad[3 + getattr(ctx, "h0_input", 1)] and len(meta) > 5
                and meta[5]):
            C_ = _native.C()
            plan_ws = torch.empty(C_.emb_det_ws_bytes(B * T, emb.shape[0], E), device=dev, dtype=torch.uint8)
        _native.C().lstm(0, ids.data_ptr(), B, T, E, H, L, C, pad_idx, emb.data_ptr(),
                         [lw[0].data_ptr() for lw in layers], [lw[1].data_ptr() for lw in layers],
                         [lw[2].data_ptr() for lw in layers], [lw[3].data_ptr() for lw in layers],
                         w_fc.data_ptr(), b_fc.data_ptr(), _native.ptr(h0c), _native.ptr(c0c), _native.ptr(pred),
                         hn.data_ptr(), cn.data_ptr(), ws.data_ptr(), 0, rng.ptr() if rng is not None else 0, salt,
                         thresh, _rng.scale(p), 0, 0, 0, 0, [], [], [], [], 0, 0, 0, 0, 0, 0,
                         emb.shape[0] if plan_ws is not None else 0, _native.ptr(plan_ws),
                         last.data_ptr(), 0, labels.data_ptr() if ce else 0, ce[0].data_ptr() if ce else 0,
                         ce[1].data_ptr() if ce else 0, ce[2].data_ptr() if ce else 0, ce[3].data_ptr() if ce else 0,
                         0, 0, int(plan_ws is not None), tick[1:].data_ptr(), _native.stream())
        # (inside Function.forward grad mode is off: the embedding's needs_input_grad says whether
        # a backward will want the table gradient; the inputs before it: ids, [labels,] h0, c0, meta;
        # meta[5]: grad mode at the call)
        ctx.emb_plan = None
        if plan_ws is not None:
            ctx.emb_plan = (plan_ws, _native.C().emb_plan_algo(B * T, emb.shape[0]))
        ctx.meta = (L, p, rng, salt, pad_idx, B, T, E, H, C)
        ctx.has_h0, ctx.has_c0 = h0 is not None, c0 is not None
        ctx.save_for_backward(ids, ws, h0c, c0c, *params)
        if ce is not None:
            ctx.ce_dlast = ce[1]
            return ce[2], last
        return pred, hn, cn, last

    @staticmethod
    def backward(ctx, dpred, dhn, dcn, dlast):
        return LSTMFn._backward(ctx, dpred, dhn, dcn, dlast, None)

    @staticmethod
    def _backward(ctx, dpred, dhn, dcn, dlast, dscale):
        """dscale: a device scalar the kernels multiply dpred by (the fused CE's dloss), or None."""
        L, p, rng, salt, pad_idx, B, T, E, H, C = ctx.meta
        ids, ws, h0c, c0c, *params = ctx.saved_tensors
        emb, layers, w_fc, b_fc = unpack(params, L)
        dev = ids.device
        # the classifier's loss reads only the last step: hand the kernel that [B, C] gradient
        # (no zero-filled [B, T, C] tensor, no scatter); a full dpred (+ dlast) takes the general path
        last_only = 0
        if dpred is None and dlast is not None:
            dpred, last_only = dlast.float().contiguous(), 1
        elif dpred is None:
            dpred = torch.zeros(B, T, C, device=dev)
        else:
            dpred = dpred.float().contiguous()
            if dlast is not None:
                dpred = dpred.clone()
                dpred[:, -1] += dlast.float()
        dhn = dhn.float().contiguous() if dhn is not None else None
        dcn = dcn.float().contiguous() if dcn is not None else None
        ws_da = torch.empty(B, L, T, 4 * H, device=dev, dtype=torch.float32)
        i0 = getattr(ctx, "h0_input", 1)  # position of h0 among the Function's inputs
        dh0 = torch.empty(L, B, H, device=dev) if ctx.needs_input_grad[i0] else None
        dc0 = torch.empty(L, B, H, device=dev) if ctx.needs_input_grad[i0 + 1] else None
        orig = params
        g = [grad_buf(t) for t in orig]
        g_emb, g_layers, g_fc, g_bfc = unpack(g, L)
        C_ = _native.C()
        slab = torch.empty(C_.lstm_slab_floats(B, E, H, L, C), device=dev, dtype=torch.float32)
        want_emb = orig[0].requires_grad
        xe = torch.empty(B, T, E, device=dev, dtype=torch.float32) if want_emb else None
        plan = getattr(ctx, "emb_plan", None) if want_emb else None
        if plan is not None:  # the forward launch ordered the ids already: sum only
            ews = plan[0]
        else:
            ews = torch.empty(C_.emb_det_ws_bytes(B * T, emb.shape[0], emb.shape[1]), device=dev,
                              dtype=torch.uint8) if want_emb else None
        _native.C().lstm(1, ids.data_ptr(), B, T, E, H, L, C, pad_idx, emb.data_ptr(),
                         [lw[0].data_ptr() for lw in layers], [lw[1].data_ptr() for lw in layers],
                         [lw[2].data_ptr() for lw in layers], [lw[3].data_ptr() for lw in layers],
                         w_fc.data_ptr(), b_fc.data_ptr(), _native.ptr(h0c), _native.ptr(c0c), 0, 0, 0,
                         ws.data_ptr(), ws_da.data_ptr(), rng.ptr() if rng is not None else 0, salt,
                         _rng.threshold(p), _rng.scale(p), dpred.data_ptr(), _native.ptr(dhn), _native.ptr(dcn),
                         g_emb.data_ptr() if orig[0].requires_grad else 0,
                         [lw[0].data_ptr() for lw in g_layers], [lw[1].data_ptr() for lw in g_layers],
                         [lw[2].data_ptr() for lw in g_layers], [lw[3].data_ptr() for lw in g_layers],
                         g_fc.data_ptr(), g_bfc.data_ptr(), _native.ptr(dh0), _native.ptr(dc0), slab.data_ptr(),
                         _native.ptr(xe), emb.shape[0], _native.ptr(ews), 0, last_only, 0, 0, 0, 0,
                         ctx.tick[8:].data_ptr(), _native.ptr(dscale), plan[1] if plan is not None else 0,
                         0, 0, _native.stream())
        ctx.emb_plan = None
        grad_ready(*orig)
        return (None, dh0 if ctx.has_h0 else None, dc0 if ctx.has_c0 else None, None) + (None,) * len(params)


_CE_TICKETS = {}
# the embedding backward's id ordering made by the forward launch (True; LSTM step 0.330 -> 0.294
# ms, docs/PERF_NOTES.md round 4) or by the backward itself (False: tests)
EMB_IN_FORWARD = True




def _ce_ticket(dev):
    """Ticket counters (zeroed once, re-armed by the kernels) for op calls without a model's own
    block (LSTM._tick): [0] the fused CE of the forward, [1] the embedding side plan, [8:] the
    backward weight-gradient kernel's (L + 1) x 8 column-tile tickets.  Shared per device: such
    calls must not run concurrently on different streams (each launch completes its ticket rounds
    before the next one on its stream starts)."""
    t = _CE_TICKETS.get(dev)
    if t is None:
        t = _CE_TICKETS[dev] = torch.zeros(8 + 8 * 5, device=dev, dtype=torch.int32)
    return t


class LSTMCEFn(torch.autograd.Function):
    """The LSTM classifier with the mean cross-entropy of its last step fused into the forward
    kernel's tail (csrc/kernels/lstm.hip lstm_ce_tail): returns (loss, pred[:, -1]); the backward
    feeds the precomputed head gradient (softmax - onehot) / B, times dloss, to the BPTT kernel."""

    @staticmethod
    def forward(ctx, ids, labels, h0, c0, meta, *params):
        ctx.h0_input = 2
        loss, last = LSTMFn._forward(ctx, ids, h0, c0, meta, params, labels)
        ctx.mark_non_differentiable(last)
        return loss, last

    @staticmethod
    def backward(ctx, dloss, dlast_unused):
        if dloss is None:
            return (None,) * (5 + len(ctx.saved_tensors) - 4)
        ds = dloss.reshape(1).float().contiguous()
        grads = LSTMFn._backward(ctx, None, None, None, ctx.ce_dlast, ds)
        return (None, None) + grads[1:3] + (None,) + grads[4:]


def lstm_classifier_ce(ids, labels, h0, c0, params, num_layers, dropout=0.0, training=True, rng=None, salt=0,
                       padding_idx=None, tick=None):
    """(mean CE of pred[:, -1] against ``labels``, pred[:, -1]) — the classifier's training loss
    (distributed_lstm.py:186-189) with the CE fused into the GPU kernel; CPU: torch reference."""
    p = dropout if training else 0.0
    emb, layers, w_fc, _ = unpack(params, num_layers)
    E, H, C = emb.shape[1], layers[0][1].shape[1], w_fc.shape[0]
    if ids.is_cuda and _native.use_native(ids) and supported(E, H, num_layers, C):
        pad = -1 if padding_idx is None else int(padding_idx)
        return LSTMCEFn.apply(ids, labels, h0, c0, (num_layers, p, rng, salt, pad, torch.is_grad_enabled(), tick),
                              *params)
    last, _, _, _ = lstm_classifier_last(ids, h0, c0, params, num_layers, dropout, training, rng, salt, padding_idx,
                                         tick)
    return torch.nn.functional.cross_entropy(last, labels), last


def lstm_classifier(ids, h0, c0, params, num_layers, dropout=0.0, training=True, rng=None, salt=0,
                    padding_idx=None, tick=None):
    """pred, h_n, c_n of embedding -> LSTM(num_layers, dropout) -> linear head (every step)."""
    p = dropout if training else 0.0
    emb, layers, w_fc, _ = unpack(params, num_layers)
    E, H, C = emb.shape[1], layers[0][1].shape[1], w_fc.shape[0]
    if ids.is_cuda and _native.use_native(ids):
        if not supported(E, H, num_layers, C):
            raise NotImplementedError(f"sparkmi LSTM kernel: unsupported shape E={E} H={H} L={num_layers} C={C} "
                                      "(H in {16,32,64}, 4*H*L <= 512, E <= 2H and <= 64, C <= 16)")
        pad = -1 if padding_idx is None else int(padding_idx)
        pred, hn, cn, _ = LSTMFn.apply(ids, h0, c0, (num_layers, p, rng, salt, pad, torch.is_grad_enabled(), tick),
                                       *params)
        return pred, hn, cn
    seed = rng.current() if (rng is not None and p > 0) else 0
    return reference_forward(ids, h0, c0, params, num_layers, p, seed, salt, padding_idx)


def lstm_classifier_last(ids, h0, c0, params, num_layers, dropout=0.0, training=True, rng=None, salt=0,
                         padding_idx=None, tick=None):
    """(pred[:, -1] contiguous, pred, h_n, c_n): the GPU kernel writes the last step's prediction
    as its own output, so a loss on it needs no slice copy and its backward no zero-filled dpred."""
    p = dropout if training else 0.0
    emb, layers, w_fc, _ = unpack(params, num_layers)
    E, H, C = emb.shape[1], layers[0][1].shape[1], w_fc.shape[0]
    if ids.is_cuda and _native.use_native(ids) and supported(E, H, num_layers, C):
        pad = -1 if padding_idx is None else int(padding_idx)
        pred, hn, cn, last = LSTMFn.apply(ids, h0, c0, (num_layers, p, rng, salt, pad, torch.is_grad_enabled(),
                                                        tick), *params)
        return last, pred, hn, cn
    pred, hn, cn = lstm_classifier(ids, h0, c0, params, num_layers, dropout, training, rng, salt, padding_idx, tick)
    return pred[:, -1, :].contiguous(), pred, hn, cn
