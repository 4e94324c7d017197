"""Native communication layer: the xGMI IPC all-reduce of sparkmi._comm.

``IpcAllReduce`` — all-reduce over IPC-mapped uncached device memory, one node, every rank
reading its peers directly over xGMI (one hop on the 7 point-to-point links) instead of a ring:
  * one-shot (buckets <= ``ONE_SHOT_MAX_BYTES`` or 2 ranks): every rank reads every peer's
    bucket and sums it — the latency path for the MLP's 256 B and the CNN's 31 KB gradients
    (distributed_multilayer_perceptron.py:103-106, distributed_cnn.py:152-156);
  * two-shot (larger buckets, e.g. the LSTM's 12.3 MB dense embedding gradient): reduce-scatter
    (rank r sums chunk r, reading its 1/w slice from all peers at once) then all-gather —
    2 (w - 1) / w of the bucket over xGMI per rank instead of (w - 1);
  * zero-copy two-shot (``register(buffer)`` + ``algo=3``): the same reduce-scatter + all-gather
    read straight out of every rank's IPC-registered gradient buffer (the flat gradient of
    sparkmi/parallel/ddp.py) — no staging copy, 2 n fewer local HBM bytes per call, one extra
    signal round so no rank's next backward overwrites a bucket a slow peer still reads.  A probed
    candidate: DataParallel measures it against the staged kernel and RCCL.
Both sum in rank order (bit-identical results on every rank) and keep their epoch on the device,
so a call can sit inside a captured HIP graph (a small model's whole data-parallel step is one
replay).  A peer that stops signalling is detected by a bounded poll: the bucket is NaN-poisoned,
a sticky device flag is set, and ``check()`` raises ``IpcPeerLost``.  Handles are exchanged once
through torch.distributed (any backend, gloo included), so two processes sharing one GPU can
exercise it too.  Bulk collectives (the transformer's 188 MB gradient) go through RCCL — torch's
"nccl" process group — in sparkmi/parallel/ddp.py.
"""
import os

import torch
import torch.distributed as dist

from .. import _native

ONE_SHOT_MAX_BYTES = 256 << 10

# IPC lifetime policy (measured, tools/zc_alloc_probe.py: 4 processes creating and closing several
# instances): once an exported allocation is freed and a new one is exported, peers can map the new
# handle to stale memory — wrong sums, sometimes only in part of the buffer.  So within a process
#  * exported staging / signal regions are never hipFree'd: they go back to _POOL (bytes ->
#    [(ptr, handle)]); a signal region is re-zeroed when handed out again (before the handle
#    exchange: no peer can signal into it earlier), a staging region is not — a slow peer may
#    still be reading the last call's chunk from it when this rank has already moved on;
#  * an allocation is exported once (_EXPORTS: allocation base -> handle), e.g. a torch gradient
#    segment registered again by a later instance;
#  * a peer handle is imported once and never closed (_IMPORTS: handle -> mapped base).
_POOL = {}
_EXPORTS = {}
_IMPORTS = {}


def _export(C, ptr):
    """(handle, byte offset of ptr in its allocation) — one export per allocation."""
    base, size = C.ipc_range(ptr)
    h = _EXPORTS.get((base, size))
    if h is None:
        h = _EXPORTS[(base, size)] = C.ipc_export(base)[0]
    return h, ptr - base


def _open(C, h):
    p = _IMPORTS.get(h)
    if p is None:
        p = _IMPORTS[h] = C.ipc_open(h)
    return p


def _alloc(C, nbytes, zero):
    free = _POOL.get(nbytes)
    if free:
        p, h = free.pop()
        if zero:
            C.ipc_memset0(p, nbytes)
        return p, h
    return C.ipc_alloc(nbytes)  # (zeroed)


class IpcUnavailable(RuntimeError):
    """IPC mapping or the all-reduce self-test failed on at least one rank (all ranks agree)."""


class IpcPeerLost(RuntimeError):
    """An IPC all-reduce timed out waiting for a peer: the bucket of that call was NaN-poisoned
    (never a finite partial sum) and the group must fail (the launcher restarts it from the last
    checkpoint)."""


class IpcAllReduce:
    """Sum-all-reduce of fp32 tensors of up to ``cap_floats`` elements among the ranks of
    ``group`` (one node), in place, on the current stream."""

    def __init__(self, cap_floats=1 << 18, group=None, blocks=None, timeout_s=None):
        C = _native.comm()
        self.C = C
        if timeout_s is None:
            timeout_s = float(os.environ.get("SPARKMI_IPC_TIMEOUT_S", "4"))
        # the kernel's poll bound: ~2^24 polls with s_sleep back-off take ~4 s
        self.spins = max(1, int(float(timeout_s) * (1 << 24) / 4.0))
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > C.IPC_MAX_RANKS:
            raise ValueError(f"IPC all-reduce supports <= {C.IPC_MAX_RANKS} ranks")
        self.cap = (int(cap_floats) + 3) // 4 * 4
        self.blocks = blocks
        # 1 | 2: every call uses that kernel (tests; SPARKMI_IPC_ALGO), else algo_for(size)
        self.force_algo = int(os.environ.get("SPARKMI_IPC_ALGO", "0")) or None
        data, hdata = _alloc(C, 2 * self.cap * 4, zero=False)
        sig, hsig = _alloc(C, C.IPC_MAX_BLOCKS * C.IPC_MAX_RANKS * 4, zero=True)
        self._own = ((2 * self.cap * 4, data, hdata), (C.IPC_MAX_BLOCKS * C.IPC_MAX_RANKS * 4, sig, hsig))
        handles = [None] * self.world
        dist.all_gather_object(handles, (hdata, hsig), group=group)
        self.data, self.sig = [], []
        opened = True
        for r, (hd, hs) in enumerate(handles):
            if r == self.rank:
                self.data.append(data)
                self.sig.append(sig)
            elif opened:
                try:
                    pd, ps = _open(C, hd), _open(C, hs)
                except RuntimeError:
                    opened = False
                    continue
                self.data.append(pd)
                self.sig.append(ps)
        self.err = torch.zeros(1, dtype=torch.int32, device="cuda")
        # {epoch, ticket, signal value, pad}: advanced by the kernels' last block
        self.ctr = torch.zeros(4, dtype=torch.int32, device="cuda")
        # every rank must be able to map every peer AND the kernel must produce the exact sum on
        # this topology (peer reads over xGMI, system-scope flags): a one-call self-test whose
        # verdict all ranks agree on through the regular process group; on failure the caller
        # keeps the RCCL path (IpcUnavailable) instead of risking a hang or a wrong gradient
        opened = self._agree(opened)  # no rank launches a test kernel its peers will not join
        ok = opened
        if opened:
            want = float(self.world * (self.world + 1) // 2)
            for algo in (1, 2):  # both kernels must produce the exact sum on this topology
                probe = torch.full((self.cap if self.cap < 4096 else 4096,), float(self.rank + 1), device="cuda")
                self(probe, algo=algo)
                torch.cuda.synchronize()
                ok = ok and bool(int(self.err.item()) == 0 and bool((probe == want).all()))
        if not self._agree(ok):
            self.close()
            raise IpcUnavailable("IPC all-reduce self-test failed on some rank; using the collective path")
        self.err.zero_()
        self._reg = None  # (registered tensor, its pointer, every rank's pointer to it)
        dist.barrier(group=group)

    def register(self, buf):
        """IPC-register ``buf`` (a contiguous fp32 CUDA tensor of the same size on every rank, e.g.
        the flat gradient buffer) for the zero-copy kernel: every rank maps every peer's copy,
        then a self-test on ``buf`` (restored afterwards) must give the exact sum on every rank.
        Collective.  Returns False (every rank agreeing) when mapping or the self-test failed."""
        C = self.C
        ok = True
        why = ""
        try:
            h = _export(C, buf.data_ptr())
        except RuntimeError as e:
            h, ok, why = None, False, f"export: {e}"
        hs = [None] * self.world
        dist.all_gather_object(hs, (h, buf.numel()), group=self.group)
        ptrs = []
        ok = ok and all(x[0] is not None and x[1] == buf.numel() for x in hs)
        if ok:
            for r, (hq, _) in enumerate(hs):
                if r == self.rank:
                    ptrs.append(buf.data_ptr())
                    continue
                try:
                    base = _open(C, hq[0])
                except RuntimeError as e:
                    ok, why = False, f"open rank {r}: {e}"
                    break
                ptrs.append(base + hq[1])
        # every rank must have mapped every peer BEFORE any rank launches the self-test kernel: a
        # rank that skipped it would leave the others' signal counters ahead of its own, and the
        # instance stays in use for the staged kernels after a failed registration
        if not self._agree(ok):
            self.register_error = why or "a peer could not export or map its buffer"
            return False
        if ok:
            # the whole buffer (a stale or partial mapping shows up somewhere in it)
            n = buf.numel() // 4 * 4
            save = buf[:n].clone()
            buf[:n].fill_(float(1 << self.rank))  # 2^rank: a wrong sum names the rank it misread
            self._reg = (buf, buf.data_ptr(), ptrs)
            self(buf[:n], algo=3)
            torch.cuda.synchronize()
            want = float((1 << self.world) - 1)
            ok = int(self.err.item()) == 0 and bool((buf[:n] == want).all())
            if not ok:
                why = (f"self-test: err={int(self.err.item())}, "
                       f"{int((buf[:n] != want).sum())}/{n} wrong (chunk starts {buf[:n:max(1, n // self.world)].tolist()}, "
                       f"want {want}); "
                       f"offsets {[x[0][1] for x in hs]}")
            dist.barrier(group=self.group)  # every peer finished its self-test reads of this buffer
            buf[:n].copy_(save)
            torch.cuda.synchronize()
        self.register_error = why
        if not self._agree(ok):
            self._reg = None
            self.err.zero_()
            return False
        self.err.zero_()
        return True

    def _agree(self, ok):
        """True on every rank iff ``ok`` on every rank (collective)."""
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32,
                            device="cuda" if dist.get_backend(self.group) == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        return bool(int(flag.item()))

    @property
    def registered(self):
        return self._reg is not None

    def algo_for(self, numel):
        """1 = one-shot, 2 = two-shot: two-shot moves 2 (w - 1) / w of the bucket per rank instead of
        (w - 1), at the price of a second signal round — worth it past the latency-bound sizes."""
        return 1 if self.world <= 2 or numel * 4 <= ONE_SHOT_MAX_BYTES else 2

    def __call__(self, t, algo=None, stream=None, sgd=None):
        """All-reduce ``t`` in place.  ``sgd`` = (params, bf16 shadow or None, lr_t, step_t, seed or
        None, grad_scale): instead of the sum, apply plain SGD with it to ``params`` (the bucket's
        parameters, same shape as ``t``), zero ``t`` and advance step_t (and the seed) — the
        optimizer launch of a data-parallel small-model step folded into the reduction."""
        algo = algo or self.force_algo or self.algo_for(t.numel())
        if (t.dtype != torch.float32 or not t.is_contiguous() or t.numel() % 4
                or (algo != 3 and t.numel() > self.cap)):
            raise ValueError("IpcAllReduce: contiguous fp32 tensor, numel % 4 == 0, <= capacity")
        if sgd is not None and algo != 1:
            raise ValueError("IpcAllReduce: the SGD epilogue is a one-shot feature")
        data = self.data
        if algo == 3:  # zero-copy: t must lie in the registered buffer (same offset on every rank)
            if self._reg is None:
                raise ValueError("IpcAllReduce: algo 3 needs a registered buffer (register())")
            reg, base, ptrs = self._reg
            off = t.data_ptr() - base
            if off < 0 or off % 16 or off + 4 * t.numel() > 4 * reg.numel():
                raise ValueError("IpcAllReduce: algo 3 reduces 16-B aligned slices of the registered buffer")
            data = [p + off for p in ptrs]
        sp = (0, 0, 0, 0, 0, 1.0)
        if sgd is not None:
            p, pbf, lr, step, seed, gscale = sgd
            sp = (p.data_ptr(), pbf.data_ptr() if pbf is not None else 0, lr.data_ptr(), step.data_ptr(),
                  seed.data_ptr() if seed is not None else 0, float(gscale))
        n4 = t.numel() // 4
        if self.blocks:
            blocks = self.blocks
        elif algo == 1:
            blocks = max(1, min(self.C.IPC_MAX_BLOCKS, (n4 + 1023) // 1024))
        else:  # >= 512 float4 of every chunk per block
            blocks = max(1, min(self.C.IPC_MAX_BLOCKS, ((n4 + self.world - 1) // self.world + 511) // 512))
        self.C.ipc_allreduce(t.data_ptr(), t.numel(), data, self.sig, self.cap, self.rank, self.ctr.data_ptr(),
                             self.err.data_ptr(), blocks, (stream or torch.cuda.current_stream()).cuda_stream,
                             self.spins, algo, *sp)
        return t

    def failed(self):
        """True once any call timed out waiting for a peer (sticky; synchronises)."""
        return bool(int(self.err.item()))

    def check(self):
        """Raise IpcPeerLost if any call timed out waiting for a peer (synchronises)."""
        if self.failed():
            raise IpcPeerLost("IPC all-reduce: a peer did not signal within the timeout; the affected gradient "
                              "bucket was NaN-poisoned")

    def close(self):
        torch.cuda.synchronize()
        for nbytes, p, h in self._own:
            _POOL.setdefault(nbytes, []).append((p, h))  # kept for the next instance (see _POOL)
        self._own = ()  # (peer imports stay mapped: _IMPORTS)
        self._reg = None
