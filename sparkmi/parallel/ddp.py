"""Synchronous data parallelism with bucketed, backward-overlapped gradient all-reduce.

This is what the reference *intended* with DDP but never executed (the raw
module was called, so gradients were never synchronised).  Design for MI355X + RCCL/xGMI:

* gradients already live in ONE flat fp32 buffer (sparkmi.utils.flat.FlatParams), laid out in
  reverse layer order, so buckets are plain contiguous slices — no pack/unpack kernels;
* a bucket's all-reduce is issued the moment its last parameter's backward kernel has been
  enqueued (ops call ``grad_ready``), on RCCL's stream, so communication of late layers runs
  under the backward of early layers.  Weight gradients that the fused ops DEFER (grouped
  weight-gradient GEMMs, LayerNorm / split-K folds, sparkmi/ops/_grad.py) are flushed early,
  per bucket: once every parameter of a bucket is queued or final, the queues are launched, the
  parameters become final and the bucket goes to RCCL — in reverse layer order, during backward;
* buckets are large (default 64 MiB): an 8-GPU ring over xGMI is per-link bandwidth bound, and
  fewer, larger collectives amortise the per-call latency;
* averaging is folded into the optimizer (``grad_scale = 1/world``) instead of a division
  pass over the buffer;
* ``zero=True`` (ZeRO-1): each bucket is REDUCE-SCATTERED instead of all-reduced — rank r owns
  piece r of every bucket — the optimizer updates only the owned pieces (compact moments,
  one multi-range launch: sparkmi.optim.adam.Adam.shard) and the updated fp32 master pieces are
  all-gathered in place; per-rank optimizer work and state drop by 1/world and the gradient
  moves (w-1)/w instead of 2(w-1)/w of the buffer before the update;
* comm path (``SPARKMI_DP_COMM`` = auto | ipc | rccl; auto by default): gradients of up to
  ``IPC_LIMIT_BYTES`` (32 MiB: the MLP's 256 B, the CNN's 31 KB, the LSTM's 12.3 MB) on one
  node go through the xGMI IPC all-reduce (csrc/comm/ipc_allreduce.hip; one-shot for buckets
  <= 256 KB, two-shot reduce-scatter + all-gather above) — no ring latency, and since it is a
  stream-ordered kernel with a device-side epoch, the whole data-parallel step (forward,
  backward, all-reduce, optimizer) is captured as ONE HIP graph (``graph_safe``).  For larger
  gradients (the transformer's 188 MB) auto MEASURES the paths at start-up on the largest
  bucket (``comm_probe``: the staged IPC two-shot vs the ZERO-COPY IPC two-shot — every rank's
  flat gradient buffer IPC-registered, peers read the buckets in place, no staging copy — vs the
  RCCL process group vs an RCCL communicator with min_ctas = 32, i.e. more rings over the 7 xGMI
  links; max over ranks, each IPC kernel also checked for an exact sum / no timeout) and keeps the
  fastest; ``SPARKMI_DP_PROBE=0`` sends them to RCCL without measuring.  Either way a bucket's
  reduction runs on a side stream (RCCL's own, or the IPC comm stream forked from the compute
  stream at launch and joined in ``finish()``), overlapped with the rest of the backward.
* ``sparse_rows={param: ids_fn or (ids_fn, cap)}`` (opt-in; SURVEY §5.8 item 5, the LSTM
  embedding of /root/reference/distributed_lstm.py:115): a table whose gradient touches only the
  step's rows is exchanged ROW-SPARSE instead of all-reduced dense — each rank de-duplicates its
  row ids (``ids_fn()``, a device sort), gathers those rows (index_select, no table copy),
  all-gathers the (ids, rows) lists and every rank sums each touched row's contributions IN RANK
  ORDER into the gradient (csrc/kernels/sparse_rows.hip on the GPU: deterministic, only the touched
  rows written; untouched rows stay zero, so any optimizer, Adam included, sees exactly the
  all-reduced gradient).  The LSTM's 12.3 MB table moves B*T*(8 + 4*D) bytes per rank instead
  (4,128 rows: 0.56 MB).  ``cap``: a fixed list length >= any rank's id count (e.g. B * max_len):
  no host sync at all; without it the ranks agree on the longest list with one small all-reduce
  read on the host each step.  Uses the process group, so a DP step with sparse rows is not a
  single-graph (``graph_safe``) step.
* optimizer per bucket (``attach_optimizer``, PER_BUCKET_OPT): an optimizer with ``step_ranges``
  (Adam/AdamW, ZeRO-1 included) updates bucket b's range (its owned piece under ZeRO-1) right after
  bucket b's reduction completed — in launch order, each behind its own RCCL work or IPC event —
  so the update of early buckets runs under the reduction of later ones; ``step()`` then updates
  the last bucket and advances the step counter once (same bias corrections: bitwise the
  one-launch update).
The CPU/gloo path runs the identical logic (multi-process CPU tests).
"""
import os

import torch
import torch.distributed as dist

from ..ops import _grad

IPC_LIMIT_BYTES = 32 << 20  # auto without a measurement: IPC kernels up to this gradient size


def choose_comm(ipc_ms, rccl_ms, rccl_mc_ms=None, ipc_zc_ms=None):
    """The auto path for a bulk gradient from a measured all-reduce of its largest bucket (max over
    ranks): 'ipc' (the staged IPC two-shot kernel), 'ipc_zc' (the zero-copy IPC two-shot, reading
    the peers' registered gradient buffers directly), 'rccl' (the process group's RCCL
    communicator) or 'rccl_mc' (an RCCL communicator created with min_ctas = 32: more channels,
    i.e. more rings over the 7 point-to-point xGMI links of a node).  The fastest wins; a tie
    prefers that order (the graph-capturable kernels first, the staged one — no peer access to
    live gradient memory — before the zero-copy one).  All run on a side stream overlapped with
    the backward, so the isolated bucket time is the right comparison.  None = path unavailable
    (not built, or it failed its NaN / timeout check)."""
    cands = [(name, ms) for name, ms in (("ipc", ipc_ms), ("ipc_zc", ipc_zc_ms), ("rccl", rccl_ms),
                                         ("rccl_mc", rccl_mc_ms)) if ms is not None]
    if not cands:
        return "rccl"
    return min(cands, key=lambda c: c[1])[0]


MIN_CTAS = 32  # RCCL channels of the multi-channel communicator the probe measures
# plain SGD applied inside the one-shot IPC all-reduce (fuse_sgd): a data-parallel small-model step
# is then the fused gradient kernel + ONE reduction-and-update launch (False: a separate SGD launch)
FUSE_SGD = True
# the optimizer per gradient bucket: finish() updates each bucket's parameters
# as soon as THAT bucket's reduction completed (RCCL work / IPC event wait), while the later buckets
# still reduce; only the last bucket's update stays behind the collective (False: one update after
# every bucket)
PER_BUCKET_OPT = True
# the zero-copy IPC two-shot (peers read each other's registered gradient buffers, no staging copy)
# is a candidate of the bulk-gradient probe (False: not registered, never measured)
ZERO_COPY = True


def multichannel_group(world, min_ctas=MIN_CTAS):
    """A new RCCL communicator over all ranks with at least ``min_ctas`` channels (CTAs), or None
    (not the nccl backend, or the option unavailable).  Collective: every rank calls it."""
    if not dist.is_initialized() or dist.get_backend() != "nccl":
        return None
    try:
        opts = dist.ProcessGroupNCCL.Options()
        opts.config.min_ctas = int(min_ctas)
        return dist.new_group(list(range(world)), backend="nccl", pg_options=opts)
    except Exception:  # noqa: BLE001 — an older RCCL / torch without the option: not a candidate
        return None


def broadcast_flat(flat, src=0, group=None):
    """Rank-0 parameter broadcast (the DDP-constructor sync of distributed.py:862-867)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(flat.master, src=src, group=group)
        flat.refresh_shadow()


def _single_node(world):
    lw = os.environ.get("LOCAL_WORLD_SIZE")
    return lw is None or int(lw) == world


class DataParallel:
    def __init__(self, flat, group=None, bucket_mb=64.0, overlap=True, broadcast=True, zero=False, ipc=None,
                 sparse_rows=None, comm=None):
        self.flat = flat
        # parameter index -> callable returning the step's touched row ids (row-sparse exchange),
        # and its optional fixed list capacity
        self._sparse, self._sparse_cap, self._sparse_pos = {}, {}, {}
        self._sparse_flags = []  # (gathered overflow flags, nrow, cap) of fixed-capacity exchanges, for check()
        for p, fn in (sparse_rows or {}).items():
            fn, cap = fn if isinstance(fn, tuple) else (fn, None)
            self._sparse[flat.index[id(p)]] = fn
            self._sparse_cap[flat.index[id(p)]] = cap
        if self._sparse and zero:
            raise ValueError("sparse_rows and zero=True do not combine (a sparse table has no owned piece)")
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.overlap = overlap
        self._limit = int(bucket_mb * (1 << 20) / 4)
        self.zero = bool(zero) and self.world > 1
        if self.zero and 64 % self.world:
            raise ValueError("zero=True needs a world size dividing 64 (buckets are 64-element aligned)")
        self.ipc = None
        self._zc = False  # buckets go through the zero-copy IPC kernel (forced, or the probe chose it)
        # comm: auto | ipc | ipc_zc (every bucket through the zero-copy kernel) | rccl
        mode = comm or os.environ.get("SPARKMI_DP_COMM", "auto")
        if mode not in ("auto", "ipc", "ipc_zc", "rccl"):
            raise ValueError(f"SPARKMI_DP_COMM={mode!r}: auto | ipc | ipc_zc | rccl")
        if mode == "ipc_zc":
            ipc = True
        if ipc is None:
            ipc = os.environ.get("SPARKMI_IPC_AR", "1") != "0" and mode != "rccl"
        # bulk gradients in auto mode: measure the paths on the largest bucket and keep the fastest
        # (SPARKMI_DP_PROBE=0: the fixed IPC_LIMIT_BYTES rule instead, the default RCCL group)
        probe = (mode == "auto" and flat.numel * 4 > IPC_LIMIT_BYTES and self.world > 1
                 and os.environ.get("SPARKMI_DP_PROBE", "1") != "0")
        if ipc and mode == "auto" and flat.numel * 4 > IPC_LIMIT_BYTES and not probe:
            ipc = False
        self._build_buckets()
        self.comm_probe = None
        # the communicator of the gradient-bucket collectives: the caller's group, or the
        # multi-channel RCCL one when the probe measured it faster
        self.bulk_group = group
        self._mc_group = None
        if (ipc and not self.zero and self.world > 1 and flat.grad.is_cuda and self.world <= 8
                and _single_node(self.world)):
            from .comm import IpcAllReduce, IpcUnavailable
            try:
                self.ipc = IpcAllReduce(cap_floats=self._ipc_capacity(), group=group)
            except IpcUnavailable:
                self.ipc = None  # every rank agreed: buckets go through the process group
        if mode == "ipc_zc":
            if self.ipc is None or not self.ipc.register(flat.grad):
                why = getattr(self.ipc, "register_error", "") if self.ipc is not None else "no IPC path"
                raise RuntimeError(f"comm='ipc_zc': the zero-copy IPC all-reduce is unavailable here "
                                   f"(rank {self.rank}: {why or 'a peer failed'})")
            self._zc = True
        if probe:
            n = max(e - s for s, e, _ in self.buckets)
            mc = multichannel_group(self.world) if group is None else None
            # the zero-copy candidate: every rank's flat gradient buffer IPC-registered (collective;
            # all ranks agree whether mapping and its self-test succeeded)
            zc = (self.ipc is not None and ZERO_COPY and self.ipc.register(flat.grad))
            ipc_ms, rccl_ms, mc_ms, zc_ms = self._probe(n, mc, zc=zc)
            choice = choose_comm(ipc_ms, rccl_ms, mc_ms, zc_ms)
            self.comm_probe = {"bucket_bytes": n * 4, "ipc_ms": ipc_ms, "ipc_zc_ms": zc_ms, "rccl_ms": rccl_ms,
                               f"rccl_min_ctas{MIN_CTAS}_ms": mc_ms, "choice": choice}
            self._zc = choice == "ipc_zc"
            if choice not in ("ipc", "ipc_zc") and self.ipc is not None:
                self.ipc.close()
                self.ipc = None
            if choice == "rccl_mc":
                self.bulk_group = self._mc_group = mc
            elif mc is not None:
                dist.destroy_process_group(mc)
        # the IPC kernels run on a comm stream forked from the compute stream at each bucket
        # launch (joined in finish()): buckets reduce while the rest of the backward runs, as
        # RCCL's do on its own stream
        self._cs = torch.cuda.Stream(device=flat.grad.device) if self.ipc is not None else None
        self._cs_used = False
        self._pending = None
        self._works = []
        self._order = []  # (bucket, completion handle) in launch order: RCCL work, IPC event or None
        self._bopt = None
        self.opt_buckets_early = 0
        self._listener = None
        self._dlistener = None
        if self.world > 1:
            if broadcast:
                broadcast_flat(flat, 0, group)
            if overlap:
                self._listener = _grad.add_listener(self._on_ready)
                self._dlistener = _grad.add_defer_listener(self._on_queued)
        self.reset()

    @property
    def comm(self):
        if self.ipc is not None:
            return "ipc_zc" if self._zc else "ipc"
        if self.world <= 1:
            return "none"
        return "rccl_mc" if self._mc_group is not None else "rccl"

    def _probe(self, n, mc=None, iters=3, zc=False):
        """(IPC two-shot ms or None, process-group ms, multi-channel RCCL ms or None, zero-copy IPC
        two-shot ms or None) of an n-float all-reduce, max over ranks.  The zero-copy kernel runs
        on the first n floats of the registered gradient buffer (restored afterwards)."""
        import time
        dev = self.flat.grad.device
        x = torch.zeros(n, dtype=torch.float32, device=dev)
        cuda = dev.type == "cuda"
        # a gloo group reduces host tensors: its flags live on the CPU
        fdev = dev if (cuda and dist.get_backend(self.group) == "nccl") else torch.device("cpu")

        def sync():
            if cuda:
                torch.cuda.synchronize(dev)

        def timed(fn):
            for _ in range(2):
                fn()
            sync()
            dist.all_reduce(torch.zeros(1, device=fdev), group=self.group)  # line the ranks up
            sync()
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            sync()
            t = torch.tensor([(time.perf_counter() - t0) / iters * 1e3], dtype=torch.float64, device=fdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            return round(float(t.item()), 3)

        ipc_ms = timed(lambda: self.ipc(x)) if self.ipc is not None else None
        zc_ms = None
        if zc:
            gz = self.flat.grad[:n]
            keep = gz.clone()  # (restored below: the probe may run on a buffer that already holds gradients)
            bad = 0.0
            try:
                zc_ms = timed(lambda: self.ipc(gz, algo=3))
                # a wrong sum must not be chosen: all-ones in, world out, on every rank
                gz.fill_(1.0)
                self.ipc(gz, algo=3)
                sync()
                bad = 0.0 if bool((gz == float(self.world)).all()) else 1.0
            finally:
                gz.copy_(keep)
            f = torch.tensor([bad], dtype=torch.float32, device=fdev)
            dist.all_reduce(f, op=dist.ReduceOp.MAX, group=self.group)
            if float(f.item()) > 0:
                zc_ms = None
        rccl_ms = timed(lambda: dist.all_reduce(x, group=self.group))
        mc_ms = timed(lambda: dist.all_reduce(x, group=mc)) if mc is not None else None
        if self.ipc is not None:
            # a peer the IPC kernels could not reach (timed-out signal rounds: sticky error) takes
            # the IPC path out of the running on EVERY rank (the error flag is agreed), instead of
            # one rank raising while the others go on
            from .comm import IpcPeerLost
            try:
                self.ipc.check()
                bad = 0.0
            except IpcPeerLost:
                bad = 1.0
            f = torch.tensor([bad], dtype=torch.float32, device=fdev)
            dist.all_reduce(f, op=dist.ReduceOp.MAX, group=self.group)
            if float(f.item()) > 0:
                ipc_ms = zc_ms = None
        return ipc_ms, rccl_ms, mc_ms, zc_ms

    def _ipc_capacity(self):
        """Staging floats for the IPC kernels: any bucket _build_buckets can cut (for any set of
        re-cuts by align_buckets) is either within the bucket limit or ONE parameter larger than
        it (a parameter is never split), so the largest of those bounds every bucket."""
        flat = self.flat
        sizes = [(flat.offsets[i + 1] if i + 1 < len(flat.params) else flat.numel) - flat.offsets[i]
                 for i in range(len(flat.params))]
        return max([min(self._limit, flat.numel)] + sizes)

    def _build_buckets(self, cuts=()):
        """Contiguous buckets of <= bucket_mb over the flat gradient buffer; a bucket never spans
        one of the parameter indices in ``cuts`` (a new bucket starts there)."""
        flat = self.flat
        self.buckets = []  # (start, end, param indices)
        cut_set = set(cuts)
        for i in getattr(self, "_sparse", ()):  # a row-sparse table is a bucket of its own
            cut_set.update((i, i + 1))
        cur, start = [], 0
        for i, p in enumerate(flat.params):
            s = flat.offsets[i]
            e = flat.offsets[i + 1] if i + 1 < len(flat.params) else flat.numel
            if cur and ((e - start) > self._limit or i in cut_set):
                self.buckets.append((start, s, cur))
                cur, start = [], s
            cur.append(i)
        if cur:
            self.buckets.append((start, flat.numel, cur))
        self.bucket_of = {}
        for b, (_, _, idx) in enumerate(self.buckets):
            for i in idx:
                self.bucket_of[i] = b

    def align_buckets(self, groups):
        """Re-cut the buckets so none mixes parameters of different ``groups`` (a list of sets of
        id(param): the gradients final after each backward piece; parameters in no group form
        the last segment)."""
        seg = []
        for p in self.flat.params:
            k = next((i for i, gset in enumerate(groups) if id(p) in gset), len(groups))
            seg.append(k)
        cuts = [i for i in range(1, len(seg)) if seg[i] != seg[i - 1]]
        self._build_buckets(cuts)
        self.reset()

    def set_overlap(self, on):
        """Enable / disable launching bucket all-reduces from inside backward (grad_ready)."""
        if on and self._listener is None and self.world > 1:
            self._listener = _grad.add_listener(self._on_ready)
            self._dlistener = _grad.add_defer_listener(self._on_queued)
        elif not on and self._listener is not None:
            _grad.remove_listener(self._listener)
            _grad.remove_defer_listener(self._dlistener)
            self._listener = self._dlistener = None
        self.overlap = bool(on)

    def reset(self):
        # gradient-readiness bookkeeping of one backward.  A parameter reused in one forward
        # (e.g. a module applied twice) reports ready / queued once per contribution: its bucket
        # may only go to the collective after the LAST one.  The first backward learns which
        # parameters are reused (no early flush or launch at all during it); afterwards buckets
        # holding a reused parameter are reduced in finish() only.
        counts = getattr(self, "_rcount", None)
        if counts is not None and self._learning and any(counts):
            self._reused = {i for i, c in enumerate(counts) if c > 1}
            self._learning = False
        self._rcount = [0] * len(self.flat.params)
        self._pending = [len(idx) for (_, _, idx) in self.buckets]
        self._unsettled = [len(idx) for (_, _, idx) in self.buckets]
        self._settled = set()
        self._launched = [False] * len(self.buckets)
        self._works = []
        self._order = []
        self.early_flushes = 0

    _learning = True
    _reused = frozenset()

    def _early_ok(self, b):
        return not self._learning and not any(i in self._reused for i in self.buckets[b][2])

    bytes_reduced = 0  # cumulative gradient bytes handed to the collectives (metrics)

    @property
    def graph_safe(self):
        """True when the gradient reduction is a plain kernel (IPC path): the whole DP step can
        be captured into one HIP graph."""
        return self.ipc is not None and not self._sparse

    def piece(self, b):
        """[start, end) of this rank's piece of bucket ``b`` (ZeRO-1 ownership)."""
        s, e, _ = self.buckets[b]
        n = (e - s) // self.world
        return s + self.rank * n, s + (self.rank + 1) * n

    def shard_ranges(self):
        return [self.piece(b) for b in range(len(self.buckets))] if self.zero else [(0, self.flat.numel)]

    def fuse_sgd(self, opt):
        """Let the gradient reduction apply ``opt`` itself when it is plain SGD (no momentum, no
        weight decay) over this buffer and the reduction is ONE bucket on the one-shot IPC kernel
        (the CNN / MLP data-parallel steps, distributed_cnn.py:149-193,
        distributed_multilayer_perceptron.py:97-145): the kernel's epilogue does sgd_kernel's update
        (csrc/comm/ipc_allreduce.hip), bitwise the separate launch.  Checked per reduction (the
        bucket layout may change after the first backward); ``last_step_fused`` tells the runner
        whether the last finish() already stepped."""
        from ..optim.sgd import SGD
        self._sgd_opt = opt if (FUSE_SGD and isinstance(opt, SGD) and not opt.momentum and not opt.weight_decay
                                and opt.flat is self.flat and opt.zero_grad_after_step) else None
        return self._sgd_opt is not None

    def _sgd_args(self, s, e):
        """The SGD epilogue arguments for bucket [s, e) when fuse_sgd applies to it, else None."""
        o = getattr(self, "_sgd_opt", None)
        if (o is None or self.ipc is None or self.zero or self._sparse or len(self.buckets) != 1
                or self.flat.planes is not None or (self.ipc.force_algo or self.ipc.algo_for(e - s)) != 1):
            return None
        sh = self.flat.shadow
        return (self.flat.master[s:e], sh[s:e] if sh is not None else None, o.lr_t, o.step_t, o.bump_seed,
                o.grad_scale)

    last_step_fused = False

    def attach_optimizer(self, opt):
        """Update each bucket's parameters as soon as its reduction completes (PER_BUCKET_OPT): for
        an optimizer over this buffer with ``step_ranges``.  Returns whether it applies."""
        self._bopt = (opt if (PER_BUCKET_OPT and self.world > 1 and hasattr(opt, "step_ranges")
                              and getattr(opt, "flat", None) is self.flat) else None)
        return self._bopt is not None

    def update_range(self, b):
        """The flat range the optimizer updates for bucket ``b`` (ZeRO-1: the owned piece)."""
        return self.piece(b) if self.zero else self.buckets[b][:2]

    def _launch(self, b):
        if self._launched[b]:
            return
        s, e, idx = self.buckets[b]
        self._launched[b] = True
        if self.flat.grad.is_cuda:
            _grad.join(self.flat.grad.device.index)  # weight grads may still be in flight on the side stream
        if len(idx) == 1 and idx[0] in self._sparse:
            self._sparse_exchange(s, e, idx[0])
            self._order.append((b, None))  # complete in the current stream's order
            return
        g = self.flat.grad[s:e]
        self.bytes_reduced += g.numel() * g.element_size()
        if self.ipc is not None:
            self._cs.wait_stream(torch.cuda.current_stream(g.device))  # the bucket's gradients are written
            sgd = self._sgd_args(s, e)
            # zero-copy for every bucket past the latency-bound one-shot sizes (at any world size: it
            # also drops the staging copy a 2-rank one-shot makes)
            from .comm import ONE_SHOT_MAX_BYTES
            zc = self._zc and sgd is None and (e - s) * 4 > ONE_SHOT_MAX_BYTES
            self.ipc(g, algo=3 if zc else None, stream=self._cs, sgd=sgd)
            self._sgd_applied = sgd is not None
            self._cs_used = True
            ev = torch.cuda.Event()
            ev.record(self._cs)
            self._order.append((b, ev))
            return
        if self.zero:
            ps, pe = self.piece(b)
            w = dist.reduce_scatter_tensor(self.flat.grad[ps:pe], g, group=self.bulk_group, async_op=True)
        else:
            w = dist.all_reduce(g, group=self.bulk_group, async_op=True)
        self._works.append(w)
        self._order.append((b, w))

    def _sparse_exchange(self, s, e, i):
        """Row-sparse reduction of parameter ``i``'s gradient (flat slice [s, e), rows of the
        parameter's first dimension): unique local row ids (sorted; duplicates -> the dummy id
        nrow), their rows gathered, an all-gather of the fixed-length (ids, rows) lists, and the
        rank-order sum of every touched row written into the gradient."""
        p = self.flat.params[i]
        nrow = p.shape[0]
        d = p.numel() // nrow
        g = self.flat.grad[s:s + p.numel()].view(nrow, d)  # (the slice may end in alignment padding)
        ids = self._sparse[i]().reshape(-1).to(device=g.device, dtype=torch.int64)
        srt = torch.sort(ids).values
        first = torch.ones_like(srt, dtype=torch.bool)
        first[1:] = srt[1:] != srt[:-1]
        uid = torch.where(first, srt, torch.full_like(srt, nrow))
        k = self._sparse_cap.get(i)
        flag = None
        if k is None:
            # ranks may hold different numbers of ids (per-batch padded lengths): the longest list
            kt = torch.tensor([uid.numel()], dtype=torch.int64, device=g.device)
            dist.all_reduce(kt, op=dist.ReduceOp.MAX, group=self.group)
            k = int(kt.item())
        else:
            # fixed capacity (no host sync): a rank over it must not leave its peers blocked in the
            # gather below — it sends its first k ids plus an overflow flag in one extra
            # slot of the id list (id nrow + 1: outside every row range, so the sums skip it), and
            # check() raises on EVERY rank once any rank's flag is set
            over = uid.numel() > k
            if over:
                uid = uid[:k]
            flag = uid.new_full((1,), nrow + 1 if over else nrow)
        if k > uid.numel():
            uid = torch.cat([uid, uid.new_full((k - uid.numel(),), nrow)])
        if flag is not None:
            uid = torch.cat([uid, flag])
            k += 1
        valid = uid < nrow
        rows = g.index_select(0, uid.clamp(max=nrow - 1)) * valid[:, None].to(g.dtype)
        # (gloo moves host tensors: device rows of a gloo group are staged through host memory)
        host = g.is_cuda and dist.get_backend(self.group) == "gloo"
        su, sr = (uid.cpu(), rows.cpu()) if host else (uid, rows)
        all_ids = su.new_empty(self.world * k)
        all_rows = sr.new_empty(self.world * k, d)
        dist.all_gather_into_tensor(all_ids, su, group=self.group)
        dist.all_gather_into_tensor(all_rows, sr, group=self.group)
        if host:
            all_ids, all_rows = all_ids.to(g.device), all_rows.to(g.device)
        from .. import _native
        if g.is_cuda and _native.use_native(g):
            pos = self._sparse_pos.get(i)
            if pos is None or pos.shape[0] < self.world * nrow:
                pos = self._sparse_pos[i] = torch.full((self.world * nrow,), -1, dtype=torch.int32, device=g.device)
            _native.C().sparse_rank_sum(all_ids.data_ptr(), all_rows.contiguous().data_ptr(), pos.data_ptr(),
                                        g.data_ptr(), self.world, k, d, nrow, _native.stream())
        else:
            # the same math in torch: touched rows zeroed, then each rank's rows added in rank order
            # (ids unique within a rank: every index_add_ is collision-free, so the order is fixed)
            touched = all_ids[all_ids < nrow]
            g.index_fill_(0, touched, 0.0)
            for r in range(self.world):
                ir = all_ids[r * k:(r + 1) * k]
                m = ir < nrow
                g.index_add_(0, ir[m], all_rows[r * k:(r + 1) * k][m])
        self.bytes_reduced += k * (8 + 4 * d)  # bytes this rank contributed
        if flag is not None:
            self._sparse_flags.append((all_ids.view(self.world, k)[:, -1], nrow, k - 1))

    def reshard_optimizer(self, opt, old_ranges):
        """Carry a sharded optimizer's moments over a bucket re-cut (the split-graph capture aligns
        buckets to backward pieces after the eager warm-up steps): every rank scatters its compact
        moments into a full-size buffer, one all-reduce assembles them, each rank keeps its new
        pieces."""
        if not self.zero:
            return
        full = torch.zeros(2, self.flat.numel, dtype=torch.float32, device=self.flat.master.device)
        o = 0
        for s, e in old_ranges:
            full[0, s:e] = opt.m[o:o + e - s]
            full[1, s:e] = opt.v[o:o + e - s]
            o += e - s
        dist.all_reduce(full, group=self.group)
        opt.shard(self.shard_ranges())
        for (s, e), off in zip(opt.ranges, opt._moff):
            opt.m[off:off + e - s] = full[0, s:e]
            opt.v[off:off + e - s] = full[1, s:e]

    def gather_params(self):
        """ZeRO-1 epilogue of a step: all-gather every bucket's updated fp32 master pieces (in
        place), refresh the bf16 shadow, and clear the gradient buffer (only the owned pieces
        were consumed by the update)."""
        if not self.zero:
            return
        m = self.flat.master
        for b in range(len(self.buckets)):
            s, e, _ = self.buckets[b]
            ps, pe = self.piece(b)
            dist.all_gather_into_tensor(m[s:e], m[ps:pe], group=self.group)
        self.flat.refresh_shadow()
        self.flat.grad.zero_()

    def launch(self, b):
        """Start bucket ``b``'s all-reduce now (idempotent within a step)."""
        self._launch(b)

    def complete_buckets(self, ready_ids):
        """Indices of the buckets whose parameters are all in ``ready_ids`` (a set of id(param))."""
        return [b for b, (_, _, idx) in enumerate(self.buckets)
                if all(id(self.flat.params[i]) in ready_ids for i in idx)]

    def _settle(self, i):
        """Count parameter ``i`` as queued-or-final; returns its bucket if that completed it."""
        if i in self._settled:
            return None
        self._settled.add(i)
        b = self.bucket_of[i]
        self._unsettled[b] -= 1
        return b if self._unsettled[b] == 0 else None

    def _on_queued(self, p):
        i = self.flat.index.get(id(p))
        if i is None or self._pending is None:
            return
        b = self._settle(i)
        if b is not None and self._pending[b] > 0 and self._early_ok(b):
            # every parameter of bucket b is queued or final: launch the queued weight-gradient
            # work now (its completion reports the parameters ready -> _on_ready launches b)
            self.early_flushes += 1
            _grad.flush_deferred()

    def _on_ready(self, p):
        i = self.flat.index.get(id(p))
        if i is None or self._pending is None:
            return
        self._rcount[i] += 1
        self._settle(i)
        b = self.bucket_of[i]
        if self._rcount[i] > 1 or not self._early_ok(b):
            return  # a reused parameter (or the learning step): the bucket waits for finish()
        self._pending[b] -= 1
        assert self._pending[b] >= 0, "gradient bucket bookkeeping went negative"
        if self._pending[b] == 0:
            self._launch(b)

    def finish(self):
        """Complete every bucket's reduction (launching any not yet issued) before the optimizer
        step.  With an attached optimizer (attach_optimizer) every bucket but the last launched is
        updated here, each right after its own reduction completed."""
        self.last_step_fused = False
        self.opt_buckets_early = 0
        if self.world <= 1:
            self.reset()
            return
        self._sgd_applied = False
        for b in range(len(self.buckets)):
            self._launch(b)
        self.last_step_fused = self._sgd_applied
        opt = None if self.last_step_fused else self._bopt
        cur = torch.cuda.current_stream(self.flat.grad.device) if self.flat.grad.is_cuda else None
        order = self._order
        for k, (b, h) in enumerate(order):
            if isinstance(h, torch.cuda.Event):
                cur.wait_event(h)
            elif h is not None:
                h.wait()
            if opt is not None and k < len(order) - 1:
                opt.step_ranges([self.update_range(b)])
                self.opt_buckets_early += 1
        if self._cs_used:
            cur.wait_stream(self._cs)
            self._cs_used = False
        self.reset()

    @property
    def grad_scale(self):
        return 1.0 / self.world

    def check(self):
        """Fail loudly if the gradient reduction lost a peer (IPC path: a poll timed out, the
        bucket was NaN-poisoned; sparkmi.parallel.comm.IpcPeerLost).  Synchronises: call it every
        log interval (Trainer) — inside a replayed HIP graph nothing else looks."""
        if self.ipc is not None:
            self.ipc.check()
        flags, self._sparse_flags = self._sparse_flags, []
        for f, nrow, cap in flags:
            if int(f.max().item()) > nrow:
                raise ValueError(f"sparse_rows: a rank's unique ids exceeded the list capacity {cap} (its gradient "
                                 f"rows past the capacity were dropped); raise sparse_cap")

    def close(self):
        if self.ipc is not None:
            self.ipc.check()
            self.ipc.close()
            self.ipc = None
        if self._mc_group is not None:
            dist.destroy_process_group(self._mc_group)
            self._mc_group = None
            self.bulk_group = self.group
        if self._listener is not None:
            _grad.remove_listener(self._listener)
            self._listener = None
        if self._dlistener is not None:
            _grad.remove_defer_listener(self._dlistener)
            self._dlistener = None
