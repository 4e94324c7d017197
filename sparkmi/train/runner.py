"""Training-step executor: eager or HIP-graph-captured, optionally data-parallel.

A "step" = dropout-seed bump -> forward -> loss -> backward (gradients land in the flat fp32
buffer) -> gradient all-reduce (data-parallel) -> fused optimizer launch.
With ``graph=True`` the step's kernels are captured once into a hipGraph after a few eager
warm-up steps and then replayed: one host launch per step instead of hundreds, which matters
at the reference's small per-GPU batches.  Inputs are copied into static
device buffers before each replay (or, with ``bind_inputs``, read in place by a graph captured per
batch when the batches live at fixed device addresses).
  * one executor: the whole step (optimizer included) is one graph;
  * data-parallel: the graph holds forward + backward; the gradient buckets are then
    all-reduced by RCCL (a few large collectives over the flat buffer) and the optimizer runs
    as one launch.  Collectives stay outside the graph, so no RCCL-in-capture dependency;
    eager data-parallel steps instead overlap the bucket all-reduces with backward.
  * data-parallel with ``split_fn`` (a loss whose autograd graph is cut into segments, e.g.
    Transformer.training_step_split at the encoder output and mid-encoder): the step is
    several graphs — G1 = forward + backward of the top segment (decoder + vocab projection),
    then one graph per lower segment's backward.  After each graph replays, the gradient
    buckets whose parameters all became final in it are all-reduced on RCCL's stream while the
    next graph replays; only the last segment's buckets are reduced after the backward.  Still
    no collective inside a graph.
"""
import torch

from ..ops import _grad
from ..ops.embedding import join_plans

# Optimizer update in two parts (single executor, an optimizer with step_ranges): the parameters
# whose gradients are final at the backward's overlapped flush (the decoder's, once the backward
# reaches the encoder: sparkmi/ops/_grad.py flush_groups_async) are updated right there on the
# side stream, behind their weight-gradient group and beside the encoder's backward; step()
# then updates the rest and advances the step counter.  Bitwise the one-launch update.
EARLY_UPDATE = True
# how many of the backward's overlapped flushes (cuts) get an early update: the second is the bf16
# step's mid-encoder flush (sparkmi/models/transformer.py ENC_MID_FLUSH_BF16)
EARLY_UPDATE_CUTS = 2
# the late cut (sparkmi/ops/_grad.py flush_deferred): the parameters the main stream finishes while
# the last group still runs on the side stream (embedding tables, LayerNorm folds) are updated there
LATE_UPDATE = True


class _EarlyUpdate:
    """Learns, on the first backward, which parameters are final at each cut (reported final
    before it, or launched by it, never reported again after it, and not in an earlier cut's
    plan), and from the next backward on updates their flat ranges at that cut (at most
    EARLY_UPDATE_CUTS cuts).  Reference: the per-step Adam of pytorch_machine_translator.py:192-196
    / distributed_lstm.py:193-195, split by readiness."""

    def __init__(self, opt):
        self.opt = opt
        self.plans = None     # per cut: (flat ranges, ids) updated at that cut
        self.begin()

    def begin(self):
        self.ready = []       # (id, number of cuts passed when it was reported)
        self.ats = []         # per cut: (ids final at it, late cut)
        self.used = []

    def on_ready(self, p):
        if _grad.CONFIRMING[0]:
            return
        self.ready.append((id(p), len(self.ats)))

    def at_cut(self, launched, late=False):
        """A side-stream cut: everything reported final so far plus the launched parameters are
        final once the side stream gets here.  The late cut (on the main stream, while a group
        still runs on the side stream): only the launched parameters are."""
        k = len(self.ats)
        at = {id(p) for p in launched} if late else {i for i, _ in self.ready} | {id(p) for p in launched}
        self.ats.append((at, late))
        if self.plans is not None and k < len(self.plans):
            rs, ids = self.plans[k]
            if rs and ids <= at:
                self.opt.step_ranges(rs)  # behind the launched work, on the stream the cut runs on
                self.used.append(k)

    def _after(self, k):
        return {i for i, c in self.ready if c > k}

    def end(self):
        if not self.ats:
            return
        if self.plans is None:
            flat = self.opt.flat
            taken, plans = set(), []
            for k, (at, late) in enumerate(self.ats):
                if not (k < EARLY_UPDATE_CUTS or (late and LATE_UPDATE)):
                    plans.append(([], set()))
                    continue
                ids = at - self._after(k) - taken
                taken |= ids
                rs = []
                for p, o in zip(flat.params, flat.offsets):
                    if id(p) in ids:
                        e = o + (p.numel() + 63) // 64 * 64
                        if rs and rs[-1][1] == o:
                            rs[-1] = (rs[-1][0], e)
                        else:
                            rs.append((o, e))
                plans.append((rs, ids))
            self.plans = plans
            return
        for k in self.used:
            if self.plans[k][1] & self._after(k):
                raise RuntimeError("early optimizer update: a parameter updated at a cut received more gradient "
                                   "after it")

    @property
    def plan(self):  # the first cut's ranges (tests / tools)
        return self.plans[0][0] if self.plans else None


class StepRunner:
    def __init__(self, model, loss_fn, optimizer, ddp=None, graph=False, warmup_eager=3, split_fn=None,
                 fused_step=None, bind_inputs=False, max_bound=32, fused_grad=None, fused_steps=None):
        self.model = model
        # bind_inputs: batches that live at fixed device addresses (an HBM-resident dataset's
        # batch views) are read IN PLACE by a graph captured per batch (shared memory pool, at
        # most max_bound of them) instead of being copied into static buffers before every
        # replay: single-executor whole-step graphs only; other modes copy as before
        self.bind_inputs = bind_inputs
        self.max_bound = max_bound
        self._bound = {}
        self._bound_pool = None
        # run_steps: ``unroll`` consecutive bound steps replay as ONE graph (each graph launch
        # costs ~8 us of device-side scheduling between replays, 12 % of a CNN step)
        self.unroll = 1
        self._multi = {}
        # fused_step(model, optimizer, *batch) -> loss or None: a whole single-executor step in
        # one kernel (e.g. MultilayerPerceptron.fused_sgd_step); None falls back to the chain
        self.fused_step = fused_step
        # fused_grad(model, *batch) -> loss or None: forward + backward in one kernel, the batch
        # gradient added to the flat gradient buffer (e.g. FashionMNISTModel.fused_grad_step); the
        # gradient reduction (data-parallel) and the optimizer follow as usual — a data-parallel
        # small-model step is then that kernel + the IPC all-reduce + the optimizer
        self.fused_grad = fused_grad
        # fused_steps(model, optimizer, batches) -> [loss per step] or None: several consecutive
        # single-executor steps in ONE kernel (e.g. MultilayerPerceptron.fused_sgd_steps), used for
        # the multi-step graphs of run_steps; None falls back to one step at a time
        self.fused_steps = fused_steps
        # pre_step(): launches that produce the step's inputs in place (e.g. DeviceLoader(fixed=
        # True).pre_step: the next shuffled batch gathered at a device cursor into the buffers the
        # step reads).  Bound / multi-step graphs capture it with the step; every other mode runs
        # it eagerly before the step (before the static-input copy of a copying graph)
        self.pre_step = None
        self._pre_inline = False
        self.last_group_sum = None  # the summed loss of the last multi-step graph replay (run_steps)
        self.loss_fn = loss_fn          # loss_fn(model, *batch) -> scalar loss tensor
        self.split_fn = split_fn        # split_fn(model, *batch) -> (loss, leaf, root), see module doc
        self.graph2 = None              # split mode: the lower segments' backward graphs
        self.bucket_waves = []          # split mode: buckets to launch after each graph
        self._split_keep = None
        self.opt = optimizer
        self.ddp = ddp
        self.graph_requested = graph
        self.warmup_eager = warmup_eager
        self.graph = None
        self.static_in = None
        self.static_loss = None
        self.steps = 0
        # per-phase device timing: HIP events around forward+backward, gradient
        # reduction and the optimizer, read back (one sync) by pop_phases() every log interval
        self.phase_timing = False
        self._phase_events = []
        self._opt_in_graph = False      # the captured graph holds the gradient reduction + optimizer
        if ddp is not None:
            optimizer.grad_scale = ddp.grad_scale
            if ddp.zero:
                if not hasattr(optimizer, "shard"):
                    raise ValueError(f"zero=True (ZeRO-1) needs an optimizer with sharded state; "
                                     f"{type(optimizer).__name__} has none (use Adam/AdamW or zero=False)")
                optimizer.shard(ddp.shard_ranges())
            elif hasattr(ddp, "fuse_sgd"):
                ddp.fuse_sgd(optimizer)  # plain SGD inside the one-shot IPC reduction, when it applies
            if hasattr(ddp, "attach_optimizer"):
                ddp.attach_optimizer(optimizer)  # the update per gradient bucket, behind its reduction

    def _opt_step(self):
        """The optimizer launch — unless the gradient reduction just applied it (ddp.fuse_sgd)."""
        if self.ddp is not None and getattr(self.ddp, "last_step_fused", False):
            return
        self.opt.step()

    @property
    def _dp(self):
        return self.ddp is not None and self.ddp.world > 1

    def _advance_seed(self):
        """The dropout step seed for this step.  The first time, where the optimizer's update kernel
        can advance it (a device seed and an optimizer with ``bump_seed``), the seed is advanced
        once here and handed to the optimizer, which advances it at the end of every step for the
        next one: one launch fewer per step, the same seed sequence.  Otherwise one bump launch."""
        rng = getattr(self.model, "rng", None)
        if rng is None:
            return
        if self.opt is not None and getattr(self.opt, "bump_seed", False) is rng.seed:
            return  # advanced by the previous step's optimizer launch
        rng.advance()
        if (hasattr(self.opt, "bump_seed") and self.opt.bump_seed is None and rng.seed.is_cuda
                and not torch.cuda.is_current_stream_capturing()):
            self.opt.bump_seed = rng.seed

    def _early_update(self):
        """The two-part optimizer update (EARLY_UPDATE), when it applies: one executor, an
        optimizer over a flat buffer with step_ranges and no sharding."""
        if not EARLY_UPDATE or self.ddp is not None or not hasattr(self.opt, "step_ranges"):
            return None
        if getattr(self.opt, "ranges", None) is not None or getattr(self.opt, "flat", None) is None:
            return None
        eu = getattr(self, "_eu", None)
        if eu is None or eu.opt is not self.opt:
            eu = self._eu = _EarlyUpdate(self.opt)
        return eu

    def _fwd_bwd(self, *batch):
        _grad.reset_deferred()  # a previous backward that raised must not leave queued work behind
        self._advance_seed()
        eu = self._early_update()
        if eu is not None:
            eu.begin()
            _grad.add_listener(eu.on_ready)
            _grad.add_cut_hook(eu.at_cut)
        try:
            loss = self.loss_fn(self.model, *batch)
            loss.backward(self._seed(loss))
            _grad.join()
            join_plans()  # a forward whose embedding backward did not run (frozen table): joined here
        finally:
            if eu is not None:
                _grad.remove_listener(eu.on_ready)
                _grad.remove_cut_hook(eu.at_cut)
        if eu is not None:
            eu.end()
        return loss.detach()

    def _seed(self, loss):
        """Persistent d(loss)/d(loss) = 1 (``backward()`` without it materialises ones_like
        every step: one fill launch inside every replayed graph)."""
        s = getattr(self, "_seed_t", None)
        if s is None or s.shape != loss.shape or s.dtype != loss.dtype or s.device != loss.device:
            s = self._seed_t = torch.ones_like(loss)
        return s

    def _refresh_inputs(self, batch):
        """Copy the step's inputs into the graph's static buffers: one multi-buffer copy launch
        on the GPU (one blit launch per input otherwise)."""
        from .. import _native
        st = self.static_in
        if (len(batch) <= 8 and all(b.is_cuda and b.is_contiguous() and b.shape == d.shape and b.dtype == d.dtype
                                    for b, d in zip(batch, st)) and _native.use_native(st[0])):
            _native.C().multi_copy([d.data_ptr() for d in st], [b.data_ptr() for b in batch],
                                   [b.numel() * b.element_size() for b in batch], _native.stream())
            return
        for dst, src in zip(st, batch):
            dst.copy_(src, non_blocking=True)

    def _event(self):
        if not self.phase_timing or not torch.cuda.is_available() or torch.cuda.is_current_stream_capturing():
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def _eager(self, *batch):
        if self._pre_inline and self.pre_step is not None:
            self.pre_step()
        if self.fused_step is not None and self.ddp is None:
            loss = self.fused_step(self.model, self.opt, *batch)
            if loss is not None:
                return loss
        e0 = self._event()
        loss = self.fused_grad(self.model, *batch) if self.fused_grad is not None else None
        if loss is None:
            loss = self._fwd_bwd(*batch)
        e1 = self._event()
        if self.ddp is not None:
            self.ddp.finish()
        e2 = self._event()
        self._opt_step()
        if self.ddp is not None:
            self.ddp.gather_params()  # ZeRO-1: all-gather the updated master pieces (no-op otherwise)
        e3 = self._event()
        if e0 is not None:
            self._phase_events.append((e0, e1, e2, e3))
        return loss

    def pop_phases(self):
        """Mean device seconds per phase over the steps since the last call: {fwd_bwd_s,
        allreduce_s, optim_s} (eager steps: events between the phases; graph steps: the step is
        captured as separate phase graphs while ``phase_timing`` is on, events between their
        replays)."""
        ev, self._phase_events = self._phase_events, []
        if not ev:
            return {}
        ev[-1][3].synchronize()
        n = len(ev)
        return {"fwd_bwd_s": sum(a.elapsed_time(b) for a, b, _, _ in ev) / n / 1e3,
                "allreduce_s": sum(b.elapsed_time(c) for _, b, c, _ in ev) / n / 1e3,
                "optim_s": sum(c.elapsed_time(d) for _, _, c, d in ev) / n / 1e3}

    def _fwd_bwd_split(self, *batch):
        _grad.reset_deferred()
        self._advance_seed()
        loss, segments = self.split_fn(self.model, *batch)
        loss.backward(self._seed(loss))
        _grad.join()
        return loss.detach(), segments

    def _capture_split(self):
        """G1 = forward + top-segment backward, then one graph per lower segment (all sharing
        G1's memory pool); records which gradient buckets are final after each graph."""
        ready = []

        def record(into):
            return _grad.add_listener(lambda p: into.add(id(p)))

        first = set()
        listener = record(first)
        g1 = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g1):
                self.static_loss, segments = self._fwd_bwd_split(*self.static_in)
                join_plans()  # embedding orderings forked in this forward, joined before G1 ends
        finally:
            _grad.remove_listener(listener)
        ready.append(first)
        graphs = [g1]
        for leaf, root in segments:
            seen = set()
            listener = record(seen)
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g, pool=g1.pool()):
                    root.backward(leaf.grad)
                    _grad.join()
            finally:
                _grad.remove_listener(listener)
            ready.append(seen)
            graphs.append(g)
        # a gradient also accumulated by a later graph is not final after an earlier one
        for i in range(len(ready)):
            for later in ready[i + 1:]:
                ready[i] -= later
        self._split_keep = segments  # later graphs read leaf.grad / roots' saved tensors at fixed addresses
        self.graph, self.graph2 = graphs[0], graphs[1:]
        old_ranges = self.ddp.shard_ranges()
        self.ddp.align_buckets(ready)
        if self.ddp.zero:
            self.ddp.reshard_optimizer(self.opt, old_ranges)
        self.bucket_waves = [self.ddp.complete_buckets(r) for r in ready]

    def _capture(self, batch):
        """Record one step into a HIP graph.  Capture only records (nothing executes), so no
        extra optimizer updates happen here: the ``warmup_eager`` eager steps before it already
        did every lazy initialisation (allocator pools, GEMM autotuning, library handles), and
        the caller replays the graph for the current step right after."""
        self.static_in = [b.clone() for b in batch]
        for s, b in zip(self.static_in, batch):
            if hasattr(b, "_smi_gather"):  # index-mode batch: the step reads the dataset itself
                s._smi_gather = b._smi_gather
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        if self._dp and self.split_fn is not None:
            self.ddp.set_overlap(False)
            self._capture_split()
            return
        if self._dp and not self.ddp.graph_safe:
            self.ddp.set_overlap(False)  # no collective may be enqueued during capture
            with torch.cuda.graph(g):
                self.static_loss = self._fwd_bwd(*self.static_in)
        elif self.phase_timing and self.fused_step is None:
            # phase-timed graph step: forward + backward, gradient reduction (IPC kernel) and the
            # optimizer as three graphs replayed back to back, events between them (one more
            # replay per phase than the single-graph step: timing, not the fastest path)
            # (single executor: no reduction phase, so no empty middle graph is captured)
            if self._dp:
                self.ddp.set_overlap(False)
                reduced0 = self.ddp.bytes_reduced  # capture records, it reduces nothing
            with torch.cuda.graph(g):
                self.static_loss = self._fwd_bwd(*self.static_in)
            self._phase_graphs = []
            fns = [lambda: self.ddp.finish()] if self._dp else [None]
            fns.append(lambda: (self._opt_step(), self.ddp.gather_params() if self._dp else None))
            for i, fn in enumerate(fns):
                if fn is None or (i == 1 and self._dp and self.ddp.last_step_fused and not self.ddp.zero):
                    self._phase_graphs.append(None)  # (the reduction graph already applied the SGD step)
                    continue
                pg = torch.cuda.CUDAGraph()
                with torch.cuda.graph(pg, pool=g.pool()):
                    fn()
                self._phase_graphs.append(pg)
            if self._dp:
                self.ddp.bytes_reduced = reduced0
            self._opt_in_graph = True
        else:
            # one executor, or data-parallel over the IPC all-reduce kernel: the WHOLE step
            # (forward, backward, gradient reduction, optimizer) is one graph
            with torch.cuda.graph(g):
                self.static_loss = self._eager(*self.static_in)
            self._opt_in_graph = True
        self.graph = g

    def _bind_ok(self):
        # data-parallel too when the reduction is a plain kernel (IPC path, ddp.graph_safe): the
        # bound / multi-step graphs then hold forward, backward, all-reduce and optimizer
        return (self.bind_inputs and (not self._dp or self.ddp.graph_safe) and self.split_fn is None
                and not self.phase_timing and not torch.cuda.is_current_stream_capturing())

    def _step_bound(self, batch):
        """Replay the graph captured for exactly these input tensors (capture it first if new);
        None when the cache is full (the caller takes the copying path)."""
        key = tuple((b.data_ptr(), tuple(b.shape), b.dtype) for b in batch)
        ent = self._bound.get(key)
        if ent is None:
            if len(self._bound) >= self.max_bound:
                return None
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            self._pre_inline = True
            reduced0 = self.ddp.bytes_reduced if self._dp else 0  # capture records, it reduces nothing
            try:
                with torch.cuda.graph(g, pool=self._bound_pool):
                    loss = self._eager(*batch)
            finally:
                self._pre_inline = False
                if self._dp:
                    self.ddp.bytes_reduced = reduced0  # the replay below counts the step
            if self._bound_pool is None:
                self._bound_pool = g.pool()
            self._opt_in_graph = True
            ent = self._bound[key] = (g, loss, batch)  # the batch stays referenced: its memory is the input
        ent[0].replay()
        if self._dp:
            self.ddp.bytes_reduced += self.ddp.flat.grad.numel() * 4
        return ent[1]

    def _step_multi(self, group, losses=None):
        """Replay the graph holding the steps of ``group`` (a list of batches) back to back,
        capturing it first if new; None when it cannot (cache full).  ``losses``: a list that
        receives every step's loss (device scalars the graph rewrites each replay)."""
        key = tuple(tuple((b.data_ptr(), tuple(b.shape), b.dtype) for b in batch) for batch in group)
        ent = self._multi.get(key)
        if ent is None:
            if len(self._multi) >= self.max_bound:
                return None
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            step_losses = []
            self._pre_inline = True
            reduced0 = self.ddp.bytes_reduced if self._dp else 0
            try:
                with torch.cuda.graph(g, pool=self._bound_pool):
                    fused = None
                    if self.fused_steps is not None and self.ddp is None and self.pre_step is None:
                        fused = self.fused_steps(self.model, self.opt, list(group))
                    if fused is not None:
                        step_losses = list(fused)
                    else:
                        for batch in group:
                            step_losses.append(self._eager(*batch))
                    # the group's summed loss inside the graph (metrics read one scalar per group);
                    # a multi-step kernel may already have written it
                    total = getattr(fused, "total", None)
                    if total is None:
                        total = torch.stack([l.detach().float().reshape(()) for l in step_losses]).sum()
            finally:
                self._pre_inline = False
                if self._dp:
                    self.ddp.bytes_reduced = reduced0
            if self._bound_pool is None:
                self._bound_pool = g.pool()
            self._opt_in_graph = True
            ent = self._multi[key] = (g, step_losses[-1], group, step_losses, total)
        ent[0].replay()
        self.last_group_sum = ent[4]
        if losses is not None:
            losses.extend(ent[3])
        self.steps += len(group)
        if self._dp:
            self.ddp.bytes_reduced += self.ddp.flat.grad.numel() * 4 * len(group)
        return ent[1]

    def run_steps(self, seq, losses=None):
        """Run one training step per batch of ``seq`` (a list of batch tuples), in order; returns
        the last loss (``losses``: a list that receives every step's loss).  With ``bind_inputs``
        and ``unroll`` > 1, each run of ``unroll`` consecutive batches replays as one multi-step
        graph (the same steps, one launch)."""
        loss, i, U = None, 0, self.unroll
        self.last_group_sum = None
        while i < len(seq):
            if (U > 1 and i + U <= len(seq) and self.graph_requested and seq[i][0].is_cuda
                    and self.steps >= self.warmup_eager and self._bind_ok()):
                out = self._step_multi(seq[i:i + U], losses)
                if out is not None:
                    loss, i = out, i + U
                    continue
            loss = self.step(*seq[i])
            if losses is not None:
                # a replayed graph returns its static loss, which the next replay of the same graph
                # (a fixed loader's batches are one key) overwrites: keep this step's value
                losses.append(loss.detach().clone() if self.graph_requested and loss.is_cuda else loss)
            i += 1
        return loss

    def step(self, *batch):
        self.steps += 1
        use_graph = self.graph_requested and batch[0].is_cuda
        if not use_graph or self.steps <= self.warmup_eager:
            if self.pre_step is not None:
                self.pre_step()
            return self._eager(*batch)
        if self._bind_ok():
            loss = self._step_bound(batch)
            if loss is not None:
                return loss
        if self.pre_step is not None:
            self.pre_step()  # the inputs in place before the static-input copy below
        if self.graph is None:
            self._capture(batch)  # then replayed below for this step
        self._refresh_inputs(batch)
        phased = getattr(self, "_phase_graphs", None)
        e0 = self._event()
        self.graph.replay()
        if phased is not None:
            e1 = self._event()
            if phased[0] is not None:
                phased[0].replay()
            e2 = self._event()
            if phased[1] is not None:
                phased[1].replay()
            e3 = self._event()
            if e0 is not None:
                self._phase_events.append((e0, e1, e2, e3))
            if self._dp:
                self.ddp.bytes_reduced += self.ddp.flat.grad.numel() * 4
            return self.static_loss
        if self.graph2 is not None:
            # after each backward piece, its final buckets go to RCCL while the next piece runs
            for g, wave in zip(self.graph2, self.bucket_waves):
                for b in wave:
                    self.ddp.launch(b)
                g.replay()
        if not self._opt_in_graph:
            # the graphs hold forward + backward only (data-parallel over RCCL, or split-graph
            # capture over either backend): reduce the remaining buckets, then the optimizer.
            # Phase events: fwd_bwd = the replays, allreduce = what finish() still waits for
            # (the part of the reduction not hidden under the backward), optim = the update
            e1 = self._event()
            if self._dp:
                self.ddp.finish()
            e2 = self._event()
            self._opt_step()
            if self._dp:
                self.ddp.gather_params()
            e3 = self._event()
            if e0 is not None:
                self._phase_events.append((e0, e1, e2, e3))
        elif self._dp:
            # the replayed graph reduced every bucket (IPC kernel): account its bytes
            self.ddp.bytes_reduced += self.ddp.flat.grad.numel() * 4
        return self.static_loss

    def check(self):
        """Raise if the data-parallel reduction lost a peer (synchronises; call per log interval)."""
        if self.ddp is not None:
            self.ddp.check()
