"""Embedding gather (+ optional positional-encoding add + dropout) and its scatter-add backward.

Reference: SentenceEmbedding (transformer.py:44-62: dropout_{0.1}(Embedding(x) + PE)) and the
LSTM's nn.Embedding(V, 32, padding_idx) (distributed_lstm.py:115).  GPU:
csrc/kernels/embedding.hip; the weight gradient is accumulated in fp32 straight into the
(flat) gradient buffer, rows equal to padding_idx receive no gradient.
"""
import math

import torch

from .. import _native
from . import rng as _rng
from ._grad import bf16_weight, grad_buf, grad_ready


def sinusoid_table(max_len: int, d_model: int) -> torch.Tensor:
    """Positional-encoding table identical to transformer.py:33-42 (interleaved sin/cos, fp32)."""
    even_i = torch.arange(0, d_model, 2).float()
    denominator = torch.pow(10000, even_i / d_model)
    position = torch.arange(max_len).reshape(max_len, 1)
    even_pe = torch.sin(position / denominator)
    odd_pe = torch.cos(position / denominator)
    return torch.stack([even_pe, odd_pe], dim=2).flatten(start_dim=1, end_dim=2)



# False: the whole ordering + sum in the backward (tests)
PLAN_AHEAD = True
_PLAN_STREAMS = {}
_PENDING = []  # forked plans not yet joined: [ws, stream, algo, joined]


def join_plans():
    """Make the current stream wait for every forked, not yet joined plan.  A caller that ends a
    HIP-graph capture before the backward that would join them (the data-parallel split-graph
    step: forward in the first graph, the encoder embedding's backward in the last) calls this
    at the end of that capture, so no capture ends with an unjoined side branch."""
    while _PENDING:
        plan = _PENDING.pop()
        if not plan[3]:
            torch.cuda.current_stream(plan[1].device).wait_stream(plan[1])
            plan[3] = True


def _join(plan):
    if not plan[3]:
        torch.cuda.current_stream(plan[1].device).wait_stream(plan[1])
        plan[3] = True
    for i, q in enumerate(_PENDING):  # by identity (the entries hold tensors)
        if q is plan:
            del _PENDING[i]
            break


def plan_backward(ids, T, pad_idx, weight):
    """Run the ordering half of the deterministic embedding backward (it depends on the ids only:
    pair-compare rank + plan, or the bucketed count / scan / place; csrc/kernels/embedding.hip
    smi_emb_plan) NOW, on a side stream forked from the current one, so that it overlaps the
    forward instead of sitting on the backward's critical path.  Returns [ws, stream, algo,
    joined]; the backward joins the stream (``_join``, once) and launches only the summing half.
    Called from inside Function.forward, only when a weight gradient will be wanted."""
    dev = ids.device
    C = _native.C()
    ws = torch.empty(C.emb_det_ws_bytes(T, weight.shape[0], weight.shape[1]), device=dev, dtype=torch.uint8)
    main = torch.cuda.current_stream(dev)
    s = _PLAN_STREAMS.get(dev)
    if s is None:
        # default priority: a high-priority stream inside the captured step moved the whole graph
        # onto three hardware queues and every kernel ran 1.5-3x slower (fp32 step 15.1 -> 22 ms)
        s = _PLAN_STREAMS[dev] = torch.cuda.Stream(device=dev)
    s.wait_stream(main)
    ws.record_stream(s)
    ids.record_stream(s)
    with torch.cuda.stream(s):
        algo = C.emb_plan(ids.data_ptr(), T, pad_idx, weight.shape[0], ws.data_ptr(), s.cuda_stream)
    plan = [ws, s, algo, False]
    _PENDING.append(plan)
    if len(_PENDING) > 64:  # forwards without a backward (grad mode on, no .backward()): bounded
        _join(_PENDING[0])
    return plan


class EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, pe, p, rng, salt, padding_idx, out_dtype, plan=False, flush_wgrad=False):
        B = ids.shape
        D = weight.shape[1]
        T = ids.numel()
        S = ids.shape[-1]
        ctx.p, ctx.rng, ctx.salt, ctx.pad = p, rng, salt, -1 if padding_idx is None else padding_idx
        ctx.flush_wgrad = flush_wgrad
        ctx.native = _native.use_native(ids)
        ids_c = ids.contiguous().to(torch.int64)
        if ctx.native:
            C = _native.C()
            f32 = out_dtype == torch.float32
            out = torch.empty(*B, D, device=ids.device, dtype=torch.float32 if f32 else torch.bfloat16)
            if pe is not None and pe.shape[0] < S:
                raise ValueError(f"sequence length {S} exceeds positional table {pe.shape[0]}")
            table = weight.detach() if f32 else bf16_weight(weight)
            args = (ids_c.data_ptr(), table.data_ptr(), _native.ptr(pe), out.data_ptr(), T, D,
                    S if pe is not None else 1, rng.ptr(), salt, _rng.threshold(p), _rng.scale(p))
            if f32:
                from . import gemm as G
                from . import planes as _pl
                # the first layer's GEMM operand, split by the same kernel (D % 32: no k padding)
                op = torch.empty(3, T, D, device=ids.device, dtype=torch.bfloat16) if (G.SP and D % 32 == 0) else None
                C.emb_fwd_f32(*args, _native.ptr(op), op.stride(0) if op is not None else 0, _native.stream())
                if op is not None:
                    _pl.attach(out, op)
            else:
                C.emb_fwd(*args, _native.stream())
            ctx.seed = 0
        else:
            x = weight.float()[ids_c]
            if pe is not None:
                x = x + pe[:S].float()
            ctx.seed = rng.current() if p > 0 else 0
            if p > 0:
                x = x * _rng.keep_mask(x.shape, p, ctx.seed, salt, x.device).to(x.dtype) * _rng.scale(p)
            out = x.to(out_dtype)
        ctx.plan = None
        if ctx.native and plan and PLAN_AHEAD and ctx.needs_input_grad[1]:  # plan: grad mode on at the call
            ctx.plan = plan_backward(ids_c, T, ctx.pad, weight)
        ctx.save_for_backward(ids_c, weight)
        return out

    @staticmethod
    def backward(ctx, dout):
        ids, weight = ctx.saved_tensors
        D = weight.shape[1]
        T = ids.numel()
        gw = grad_buf(weight)
        if ctx.native:
            C = _native.C()
            if ctx.flush_wgrad:
                # the last op of the backward (the encoder's embedding): every weight gradient
                # queued so far is final, so the grouped launch starts now on the side stream and
                # runs beside this sum instead of after it
                from . import _grad as _g
                _g.flush_groups_async(dout.device)
            dout = dout.contiguous()
            V = weight.shape[0]
            # deterministic backward (bit-reproducible, no float atomics): the ordering ran beside
            # the forward (plan_backward); join it and sum
            plan, ctx.plan = ctx.plan, None
            rng, salt, pad, p = ctx.rng, ctx.salt, ctx.pad, ctx.p

            def run():
                if plan is not None:
                    _join(plan)
                    C.emb_sum(plan[2], int(dout.dtype != torch.float32), ids.data_ptr(), dout.data_ptr(), gw.data_ptr(),
                              T, D, pad, rng.ptr(), salt, _rng.threshold(p), _rng.scale(p), V, plan[0].data_ptr(),
                              _native.stream())
                else:
                    bwd = C.emb_bwd_f32 if dout.dtype == torch.float32 else C.emb_bwd
                    ws = torch.empty(C.emb_det_ws_bytes(T, V, D), device=dout.device, dtype=torch.uint8)
                    bwd(ids.data_ptr(), dout.data_ptr(), gw.data_ptr(), T, D, pad, rng.ptr(), salt,
                        _rng.threshold(p), _rng.scale(p), V, ws.data_ptr(), _native.stream())
                    run.ws = ws  # held with the launch's operands
            # the table's gradient is read by nothing but the optimizer: at the end of the backward
            # when an overlapped weight-gradient group is in flight (the decoder's embedding, after
            # the cross-attention projection's backward), else now
            from . import _grad as _g
            if not ctx.flush_wgrad and _g.defer_late(dout.device, run, (weight,), hold=(dout, ids, plan)):
                return None, None, None, None, None, None, None, None, None, None
            run()
        else:
            g = dout.float()
            if ctx.p > 0:
                g = g * _rng.keep_mask(g.shape, ctx.p, ctx.seed, ctx.salt, g.device).to(g.dtype) * _rng.scale(ctx.p)
            g = g.reshape(T, D)
            idf = ids.reshape(T)
            if ctx.pad >= 0:
                keep = idf != ctx.pad
                g, idf = g[keep], idf[keep]
            gw.index_add_(0, idf, g)
        grad_ready(weight)
        return None, None, None, None, None, None, None, None, None, None


def embedding(ids, weight, pe=None, p=0.0, rng=None, salt=0, padding_idx=None, out_dtype=torch.float32,
              flush_wgrad=False):
    """``flush_wgrad``: this embedding's backward is the last op of the backward pass (the
    encoder's token embedding): it launches the queued grouped weight gradients first."""
    if rng is None:
        from .layernorm import _NULL_RNG
        rng, p = _NULL_RNG, 0.0
    return EmbeddingFn.apply(ids, weight, pe, float(p), rng, int(salt), padding_idx, out_dtype, torch.is_grad_enabled(),
                             bool(flush_wgrad))
