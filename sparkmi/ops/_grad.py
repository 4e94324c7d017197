"""Parameter-gradient plumbing shared by every fused op.

sparkmi's fused autograd Functions do not hand weight gradients back to autograd; their
backward kernels accumulate them straight into ``param.grad`` (an fp32 view into the model's
flat gradient buffer when the model was flattened by :class:`sparkmi.utils.flat.FlatParams`),
then call :func:`grad_ready` so the data-parallel engine can launch the all-reduce of a
gradient bucket as soon as its last parameter is final (overlap with the rest of backward).
"""
import contextlib
import os

import torch

_listeners = []

# ---- weight-gradient side stream ---------------------------------------------------------
# A linear layer's weight gradient (dW = dY^T X, plus the bias column sum) is off the critical
# path of backward: only dX feeds the next op.  The fused ops enqueue those GEMMs on a second
# HIP stream so they run concurrently with the dgrad / attention / norm kernels of the layers
# below (each of those GEMMs alone leaves most of the chip waiting on memory at these sizes).
# Inside a HIP-graph capture the fork/join becomes parallel graph branches.  The main stream
# joins the side stream before anything reads the gradients: at the end of every backward pass
# (autograd final callback), before a data-parallel bucket all-reduce, and before the optimizer.
# OFF by default (SPARKMI_WGRAD_STREAM=1 enables it): measured on MI355X, a replayed graph with
# the fork/join branches leaves the GPU idle 15-20 us at each cross-queue dependency (1.06 ms of
# idle per transformer step in 108 such gaps) — more than the overlap wins; the single-stream
# step has no idle gaps at all (profiles/timeline_*).
_SIDE_ENABLED = False
_side_streams = {}
_pending = {}  # device -> the stream the side work was forked from (and must be joined back into)


def _side_stream(device):
    s = _side_streams.get(device)
    if s is None:
        s = torch.cuda.Stream(device=device)
        _side_streams[device] = s
    return s


def join(device=None):
    """Make the stream the side work was forked from wait for the side stream (all devices if None).

    The join target is the RECORDED fork stream, not the caller's current stream: the autograd
    final callback may run on an engine thread whose current stream is not the backward's (during
    a graph capture that would leave the side branch unjoined)."""
    devs = list(_pending) if device is None else [device]
    for d in devs:
        main = _pending.pop(d, None)
        if main is not None:
            main.wait_stream(_side_streams[d])


@contextlib.contextmanager
def side(device, *tensors):
    """Run the enclosed launches on the weight-gradient side stream of ``device``."""
    if not _SIDE_ENABLED or device.type != "cuda":
        yield
        return
    dev = device.index if device.index is not None else torch.cuda.current_device()
    main = torch.cuda.current_stream(dev)
    s = _side_stream(dev)
    s.wait_stream(main)
    for t in tensors:
        if t is not None:
            t.record_stream(s)
    if dev not in _pending:
        _pending[dev] = main
        try:
            torch.autograd.Variable._execution_engine.queue_callback(lambda: join(dev))
        except RuntimeError:
            pass  # not inside a backward pass: callers join explicitly
    with torch.cuda.stream(s):
        yield


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



class SharedGrad:
    """Gradient buffer of a tensor whose consumers write their slices of dX in place (and return
    None to autograd): the producer's backward then reads the whole gradient at once, e.g. one
    dgrad GEMM over the six decoder kv projections (ops.linear.concat_linear)."""

    __slots__ = ("buf", "planes", "planes_only")

    def __init__(self):
        self.buf = None
        self.planes = None
        self.planes_only = False  # every writer wrote planes only (sparkmi/ops/planes.py)

    def get(self, like: torch.Tensor) -> torch.Tensor:
        if self.buf is None:
            self.buf = torch.empty_like(like)
        return self.buf

    def get_planes(self, buf: torch.Tensor) -> torch.Tensor:
        """bf16 split planes [3, rows, W] of the buffer (fp32 path), filled by the same writers;
        attached to the buffer on take() for the producer's split-plane GEMMs."""
        if self.planes is None:
            W = buf.shape[-1]
            self.planes = torch.empty(3, buf.numel() // W, W, device=buf.device, dtype=torch.bfloat16)
        return self.planes

    def take(self):
        b, self.buf = self.buf, None
        p, self.planes = self.planes, None
        only, self.planes_only = self.planes_only, False
        if b is not None and p is not None:
            from . import planes as _pl
            _pl.attach(b, p)
            b._smi_planes_only = only
        return b


class ResidualGrad:
    """Routes a residual branch's gradient into the dgrad GEMM of the sibling consumer.

    In a post-LN block ``y = LN(dropout(F(x)) + x)`` the block input ``x`` feeds both the first
    linear of F and the residual.  Autograd would add the two gradients with a separate
    elementwise pass; instead the LayerNorm backward (which always runs first) parks the
    residual gradient here and the linear's backward adds it in its dgrad epilogue (the
    ``resid`` term of the GEMM), so dX leaves the GEMM complete.
    """

    __slots__ = ("grad",)

    def __init__(self):
        self.grad = None

    def take(self):
        g, self.grad = self.grad, None
        return g


# ---- deferred LayerNorm dgamma/dbeta folds ----
# Each LayerNorm backward leaves per-block partial rows; instead of one small fold launch per
# LayerNorm (30 per transformer step, ~5 us each), the folds are queued and run as ONE batched
# launch at the end of the backward (autograd final callback), after which the parameters are
# reported ready (DDP bucket hooks / split-graph ready sets see them at the end of their
# backward piece).  SPARKMI_LN_DEFER=0 restores the per-LayerNorm fold.
LN_DEFER = True
_ln_queue = []
_cb = [False]


def _queue_flush():
    """Schedule the end-of-backward flush once per backward.  The flag is set only after the
    callback is registered; outside a backward pass (no engine to call back) flush now."""
    if not _cb[0]:
        try:
            torch.autograd.Variable._execution_engine.queue_callback(flush_deferred)
        except RuntimeError:
            flush_deferred()
            return
        _cb[0] = True


# Listeners told when a parameter's gradient is QUEUED (not yet final): the data-parallel engine
# flushes the queues early once every parameter of a gradient bucket is queued or final, so that
# bucket's all-reduce starts during the backward instead of after it (sparkmi/parallel/ddp.py).
_defer_listeners = []


def add_defer_listener(fn):
    _defer_listeners.append(fn)
    return fn


def remove_defer_listener(fn):
    if fn in _defer_listeners:
        _defer_listeners.remove(fn)


def _queued(params):
    for fn in list(_defer_listeners):
        for p in params:
            if p is not None:
                fn(p)


def pending():
    """True when deferred work is queued or a flush is scheduled."""
    return bool(_cb[0] or _ln_queue or _fold_queue or _group_queue or _late or _async["main"] is not None)


def reset_deferred():
    """Drop stale deferred state before a new backward.  A backward that raised after queueing
    work leaves the queues filled and the flush flag set (autograd discards its final callbacks);
    without this reset every later backward would queue work that is never flushed."""
    stale = pending()
    if _async["main"] is not None:
        _join_async()
    _ln_queue.clear()
    _fold_queue.clear()
    _group_queue.clear()
    _group_bytes.clear()
    _late.clear()
    _cb[0] = False
    return stale


def defer_ln_fold(part_g, part_b, nb, D, gg, gb, params, stream):
    _ln_queue.append((part_g, part_b, nb, D, gg, gb, params, stream))
    _queue_flush()
    _queued(params)


# ---- deferred split-K weight-gradient folds ----
# Same idea for the split-K slabs of the weight-gradient GEMMs (sparkmi/ops/gemm.py:wgrad):
# one fold launch per Linear (66 per transformer step) becomes one batched launch per backward
# piece; the slabs stay alive until then.  SPARKMI_FOLD_DEFER=0 folds each GEMM immediately.
FOLD_DEFER = True
_fold_queue = []


def defer_wgrad_fold(slab, splits, n, gw, nb, gb, params, stream):
    _fold_queue.append((slab, splits, n, gw, nb, gb, params, stream))
    _queue_flush()
    _queued(params)


# ---- grouped weight-gradient GEMMs ----
# A Linear's weight gradient is off the critical path of the backward (only dX feeds the next
# op), so instead of one split-K GEMM per Linear (8-16 k-steps per tile, fp32 slabs, a fold)
# every wgrad is queued here and the whole backward's wgrads run as ONE grouped launch at its
# end (csrc/kernels/gemm.hip:gemm_wgrad_group_kernel: no split-K, each tile reduces all tokens
# and adds into the fp32 gradient).  The queued dY / X stay referenced until then (autograd
# then never accumulates into them in place).  SPARKMI_WGRAD_GROUP=0 restores per-Linear GEMMs.
WGRAD_GROUP = True
_group_queue = []
GROUP_MAX = 40  # csrc/kernels/gemm.hip WG_MAX


# Memory bound of the queue: every queued dY / X stays alive until the flush (autograd would
# free dY layer by layer).  Past SPARKMI_WGRAD_GROUP_MB of distinct queued operand bytes the
# queues are flushed from inside the op (the same early flush the data-parallel engine does per
# bucket), so deep / long-sequence models keep a bounded backward peak.
GROUP_CAP_BYTES = int(float(os.environ.get("SPARKMI_WGRAD_GROUP_MB", "8192")) * (1 << 20))
_group_bytes = {}


def queued_bytes():
    return sum(_group_bytes.values())


def defer_wgrad_group(dy, x, gw, gb, params, stream):
    _group_queue.append((dy, x, gw, gb, params, stream))
    for t in (dy, x):
        _group_bytes[t.data_ptr()] = t.numel() * t.element_size()
    _queue_flush()
    _queued(params)
    if sum(_group_bytes.values()) > GROUP_CAP_BYTES:
        flush_deferred()


def _kind(e):
    """Operand format of a queued wgrad: 'planes' (fp32 as [3, T, ld] bf16 split planes), 'bf16', 'f32'."""
    return "planes" if e[0].dim() == 3 else ("bf16" if e[0].dtype == torch.bfloat16 else "f32")


def _launch_group(C, batch, st):
    kind = _kind(batch[0])
    if kind == "planes":
        C.gemm_sp_wgrad_group([b[0].data_ptr() for b in batch], [b[0].stride(1) for b in batch],
                              [b[0].stride(0) for b in batch], [b[1].data_ptr() for b in batch],
                              [b[1].stride(1) for b in batch], [b[1].stride(0) for b in batch],
                              [b[2].data_ptr() for b in batch],
                              [b[3].data_ptr() if b[3] is not None else 0 for b in batch],
                              [b[2].shape[0] for b in batch], [b[2].shape[1] for b in batch],
                              [b[0].shape[1] for b in batch], st)
        return
    fn = C.gemm_wgrad_group if kind == "bf16" else C.gemm_f32_wgrad_group
    fn([b[0].data_ptr() for b in batch], [b[0].stride(0) for b in batch],
       [b[1].data_ptr() for b in batch], [b[1].stride(0) for b in batch],
       [b[2].data_ptr() for b in batch],
       [b[3].data_ptr() if b[3] is not None else 0 for b in batch],
       [b[2].shape[0] for b in batch], [b[2].shape[1] for b in batch],
       [b[0].shape[0] for b in batch], st)


def _flush_groups(C, gq):
    by_stream = {}
    for e in gq:
        by_stream.setdefault(e[5], []).append(e)
    for st, es in by_stream.items():
        batch, outs = [], set()
        for e in es + [None]:
            # one batch's tiles run concurrently and add without atomics: outputs must be distinct;
            # a batch holds one operand format
            if e is None or len(batch) == GROUP_MAX or e[2].data_ptr() in outs or (
                    e[3] is not None and e[3].data_ptr() in outs) or (batch and _kind(e) != _kind(batch[0])):
                if batch:
                    _launch_group(C, batch, st)
                batch, outs = [], set()
            if e is not None:
                batch.append(e)
                outs.add(e[2].data_ptr())
                if e[3] is not None:
                    outs.add(e[3].data_ptr())


def _flush_ln(C, lq):
    by_stream = {}
    for e in lq:
        by_stream.setdefault(e[7], []).append(e)
    for st, es in by_stream.items():
        batch, outs = [], set()
        for e in es + [None]:
            # a batch's blocks add into their outputs without atomics: a LayerNorm used twice in
            # one backward (same gamma/beta) must land in different launches
            if e is None or len(batch) == 32 or e[4].data_ptr() in outs or e[5].data_ptr() in outs:
                if batch:
                    C.ln_bwd_reduce_multi([b[0].data_ptr() for b in batch], [b[1].data_ptr() for b in batch],
                                          [b[4].data_ptr() for b in batch], [b[5].data_ptr() for b in batch],
                                          [b[2] for b in batch], [b[3] for b in batch], 1, st)
                batch, outs = [], set()
            if e is not None:
                batch.append(e)
                outs.add(e[4].data_ptr())
                outs.add(e[5].data_ptr())


def _flush_folds(C, fq):
    by_stream = {}
    for e in fq:
        by_stream.setdefault(e[7], []).append(e)
    for st, es in by_stream.items():
        batch, outs = [], set()
        for e in es + [None]:
            # a batch's outputs must be distinct (its blocks run concurrently)
            if e is None or len(batch) == 64 or e[3].data_ptr() in outs or (
                    e[5] is not None and e[5].data_ptr() in outs):
                if batch:
                    C.splitk_fold_multi([b[0].data_ptr() for b in batch], [b[3].data_ptr() for b in batch],
                                        [b[5].data_ptr() if b[5] is not None else 0 for b in batch],
                                        [b[2] for b in batch], [b[4] for b in batch], [b[1] for b in batch], st)
                batch, outs = [], set()
            if e is not None:
                batch.append(e)
                outs.add(e[3].data_ptr())
                if e[5] is not None:
                    outs.add(e[5].data_ptr())


# ---- overlapped weight-gradient group ----
# The queued weight gradients of the part of the backward that is already done (the decoder's,
# once the backward reaches the encoder) do not depend on anything that follows, so they can run
# on a side stream while the rest of the backward runs: compute-bound wgrad tiles fill the CUs
# the bandwidth-bound LayerNorms and the latency-bound attention kernels leave idle.  ONE fork
# and ONE join per backward (a side stream per Linear cost 15-20 us per cross-queue dependency,
# see _SIDE_ENABLED above).  The launched operands stay referenced until the join; their
# parameters are reported final only after it.  Single-process only (no defer listeners: the
# data-parallel engine runs its own early flushes).  False disables it.  A flush per layer (each
# encoder / decoder layer's wgrads launched when its backward is done) measured +1.1 / +1.5 ms per
# fp32 step (profiles/r5_ab_wgrad_flush_points.log): the side-stream wgrad workgroups (one per CU,
# 147 KiB of LDS) take CUs from the critical dgrad chain.
WGRAD_OVERLAP = True
_async = {"main": None, "dev": None, "hold": [], "hold_ln": []}
# defer_late(): gradient-only launches issued while an overlapped flush is in flight run at the end
# of the backward (False: in place)
LATE_GRADS = True
_late = []

# ---- the cut: work launched at the overlapped flush ------------------------------------------
# Cut hooks run on the side stream right after the overlapped flush has launched the queued
# weight gradients (and, when a hook is registered, the queued LayerNorm folds): fn(launched
# params).  Everything reported final before the cut plus the launched parameters are final once
# the side stream reaches the hook's launches — the training-step runner updates them there
# (sparkmi/train/runner.py _EarlyUpdate: the decoder's Adam beside the encoder's backward).
# CONFIRMING[0] is True while flush_deferred reports the cut's held parameters final (after the
# join): a listener that tracks when gradients become final can tell those reports apart.
_cut_hooks = []
CONFIRMING = [False]


def add_cut_hook(fn):
    _cut_hooks.append(fn)
    return fn


def remove_cut_hook(fn):
    if fn in _cut_hooks:
        _cut_hooks.remove(fn)


def flush_groups_async(device):
    """Launch the queued grouped weight-gradient GEMMs now on the side stream of ``device``."""
    if not (WGRAD_OVERLAP and WGRAD_GROUP and _group_queue) or _defer_listeners or device.type != "cuda":
        return False
    from .. import _native
    dev = device.index if device.index is not None else torch.cuda.current_device()
    if _async["main"] is not None and _async["dev"] != dev:
        return False
    gq = list(_group_queue)
    _group_queue.clear()
    _group_bytes.clear()
    hooks = list(_cut_hooks)
    lq = list(_ln_queue) if hooks else []  # with a hook: the LayerNorm folds so far go out too
    if lq:
        _ln_queue.clear()
    main = torch.cuda.current_stream(dev)
    side = _side_stream(dev)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        st = _native.stream()
        C = _native.C()
        _flush_groups(C, [e[:5] + (st,) for e in gq])
        if lq:
            _flush_ln(C, [e[:7] + (st,) for e in lq])
        if hooks:
            launched = [p for e in gq for p in e[4] if p is not None] + [p for e in lq for p in e[6] if p is not None]
            for fn in hooks:
                fn(launched)
    if _async["main"] is None:
        _async["main"], _async["dev"] = main, dev
    _async["hold"].extend(gq)
    _async["hold_ln"].extend(lq)
    _queue_flush()  # the end-of-backward flush joins the side stream
    return True


def defer_late(device, fn, params, hold=()):
    """Defer ``fn`` (launches that only produce parameter gradients, e.g. an embedding table's
    gradient sum) to the end of the backward when an overlapped flush is in flight on ``device``:
    run in place, right after the flush, it sat on the main stream ahead of the rest of the
    backward, starved of CUs by the weight-gradient group (a 50 us sum took 460 us on the bf16
    step's critical path); at the end it runs beside the last group instead.  (A fork onto another
    stream did not help: in the replayed graph the fork landed on the main branch's queue.)
    ``params`` are reported final after it; ``hold`` keeps the operands alive.  Returns False
    (nothing deferred) otherwise: the caller runs ``fn`` now."""
    if _async["main"] is None or device.type != "cuda" or not LATE_GRADS:
        return False
    _late.append((fn, tuple(params), tuple(hold)))
    return True


def _join_async():
    """Join the overlapped flush's side stream; returns its held (group entries, LayerNorm fold
    entries)."""
    main = _async["main"]
    if main is None:
        return [], []
    main.wait_stream(_side_streams[_async["dev"]])
    held, held_ln = _async["hold"], _async["hold_ln"]
    _async["main"], _async["dev"], _async["hold"], _async["hold_ln"] = None, None, [], []
    return held, held_ln


def flush_deferred():
    """Launch every queued weight-gradient GEMM / fold, then report the parameters final.
    The queues are emptied first (try/finally): a launch that raises leaves no stale entries."""
    from .. import _native
    gq, lq, fq = list(_group_queue), list(_ln_queue), list(_fold_queue)
    late = list(_late)
    _group_queue.clear()
    _group_bytes.clear()
    _ln_queue.clear()
    _fold_queue.clear()
    _late.clear()
    _cb[0] = False
    for fn, _, _ in late:  # deferred gradient-only work: beside the still-running side-stream group
        fn()
    # launched before the join when no output is one an overlapped group (still running on the
    # side stream) writes: they then run beside it
    side_out = {t.data_ptr() for e in _async["hold"] for t in (e[2], e[3]) if t is not None}
    side_out |= {t.data_ptr() for e in _async["hold_ln"] for t in (e[4], e[5])}
    early = not side_out.intersection(t.data_ptr() for e in gq + lq + fq for t in (e[2], e[3], e[4], e[5])
                                      if isinstance(t, torch.Tensor))
    held, held_ln = ([], []) if early else _join_async()
    if gq or lq or fq:
        C = _native.C()
        _flush_groups(C, gq)
        _flush_ln(C, lq)
        _flush_folds(C, fq)
    # the LATE cut: with an overlapped group still running on the side stream, the parameters whose
    # gradients the main stream has just finished (deferred sums, LayerNorm / split-K folds) are
    # handed to the cut hooks on the main stream, ahead of the join (runner._EarlyUpdate updates
    # them there, beside the group); their reports below are then confirmations
    late_cut = early and _async["main"] is not None and bool(_cut_hooks)
    if late_cut:
        done = ([p for _, ps, _ in late for p in ps] + [p for e in lq for p in e[6] if p is not None]
                + [p for e in fq for p in e[6] if p is not None])
        if done:
            for fn in list(_cut_hooks):
                fn(done, late=True)
        else:
            late_cut = False
    if early:
        held, held_ln = _join_async()
    CONFIRMING[0] = True
    try:
        for e in held:  # overlapped groups: joined into the main stream, now final
            grad_ready(*e[4])
        for e in held_ln:
            grad_ready(*e[6])
        if late_cut:
            _report_main(lq, late, fq)
    finally:
        CONFIRMING[0] = False
    if not late_cut:
        _report_main(lq, late, fq)
    for e in gq:
        grad_ready(*e[4])


def _report_main(lq, late, fq):
    for e in lq:
        grad_ready(*e[6])
    for _, ps, _ in late:
        grad_ready(*ps)
    for e in fq:
        grad_ready(*e[6])

