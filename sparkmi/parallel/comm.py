"""Native communication layer: sparkmi._comm from Python.

``NativeComm`` — an RCCL communicator owned by sparkmi (not torch's process group): bootstrapped
from an ncclUniqueId published by rank 0 through the job's c10d TCPStore (the same rendezvous the
reference's ``init_process_group`` used, distributed_cnn.py:152), collectives on raw device
pointers on the current HIP stream, and ``abort()`` for the failure path.

``IpcAllReduce`` — one-shot all-reduce over IPC-mapped uncached device memory for
latency-bound buckets (< ~256 KB: the MLP's 256 B, the CNN's 31 KB gradients,
distributed_multilayer_perceptron.py:103-106, distributed_cnn.py:152-156): every rank reads every
peer's bucket directly over xGMI in one hop and sums in rank order (bit-identical results on
every rank).  The epoch counter lives on the device, so the call can sit inside a captured HIP
graph (the small models' whole data-parallel step is one replay).  Handles are exchanged once through torch.distributed (any backend, gloo included),
so two processes sharing one GPU can exercise it too.
"""
import torch
import torch.distributed as dist

from .. import _native

_DT = {torch.float32: "float32", torch.bfloat16: "bfloat16", torch.float16: "float16", torch.int32: "int32",
       torch.int64: "int64", torch.uint8: "uint8"}


def _store():
    return dist.distributed_c10d._get_default_store()


class NativeComm:
    def __init__(self, rank=None, world=None, device=None, store=None, tag="sparkmi_rccl"):
        init = dist.is_available() and dist.is_initialized()
        self.rank = (dist.get_rank() if init else 0) if rank is None else rank
        self.world = (dist.get_world_size() if init else 1) if world is None else world
        dev = torch.cuda.current_device() if device is None else device
        C = _native.comm()
        if self.world == 1:
            uid = C.unique_id()
        else:
            st = store if store is not None else _store()
            key = f"{tag}_uid"
            if self.rank == 0:
                st.set(key, C.unique_id())
            uid = st.get(key)
        self.comm = C.Comm(uid, self.rank, self.world, dev)

    @staticmethod
    def _s():
        return torch.cuda.current_stream().cuda_stream

    def all_reduce(self, t, op="sum"):
        self.comm.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype], op, self._s())
        return t

    def reduce_scatter(self, out, inp, op="sum"):
        self.comm.reduce_scatter(inp.data_ptr(), out.data_ptr(), out.numel(), _DT[out.dtype], op, self._s())
        return out

    def all_gather(self, out, inp):
        self.comm.all_gather(inp.data_ptr(), out.data_ptr(), inp.numel(), _DT[inp.dtype], self._s())
        return out

    def broadcast(self, t, root=0):
        self.comm.broadcast(t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype], root, self._s())
        return t

    def async_error(self):
        return self.comm.async_error()

    def abort(self):
        self.comm.abort()

    def destroy(self):
        self.comm.destroy()


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
            import os
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
        data, hdata = C.ipc_alloc(2 * self.cap * 4)
        sig, hsig = C.ipc_alloc(C.IPC_MAX_BLOCKS * C.IPC_MAX_RANKS * 4)
        self._own = (data, sig)
        handles = [None] * self.world
        dist.all_gather_object(handles, (hdata, hsig), group=group)
        self.data, self.sig, self._opened = [], [], []
        opened = True
        for r, (hd, hs) in enumerate(handles):
            if r == self.rank:
                self.data.append(data)
                self.sig.append(sig)
            elif opened:
                try:
                    pd, ps = C.ipc_open(hd), C.ipc_open(hs)
                except RuntimeError:
                    opened = False
                    continue
                self._opened += [pd, ps]
                self.data.append(pd)
                self.sig.append(ps)
        self.err = torch.zeros(1, dtype=torch.int32, device="cuda")
        self.ctr = torch.zeros(2, dtype=torch.int32, device="cuda")  # {epoch, ticket}: advanced by the kernel
        # every rank must be able to map every peer AND the kernel must produce the exact sum on
        # this topology (peer reads over xGMI, system-scope flags): a one-call self-test whose
        # verdict all ranks agree on through the regular process group; on failure the caller
        # keeps the RCCL path (IpcUnavailable) instead of risking a hang or a wrong gradient
        ok = opened
        if opened:
            probe = torch.full((self.cap if self.cap < 4096 else 4096,), float(self.rank + 1), device="cuda")
            self(probe)
            torch.cuda.synchronize()
            want = float(self.world * (self.world + 1) // 2)
            ok = bool(int(self.err.item()) == 0 and bool((probe == want).all()))
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32,
                            device="cuda" if dist.get_backend(group) == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        if not int(flag.item()):
            self.close()
            raise IpcUnavailable("IPC all-reduce self-test failed on some rank; using the collective path")
        self.err.zero_()
        dist.barrier(group=group)

    def __call__(self, t):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() % 4 or t.numel() > self.cap:
            raise ValueError("IpcAllReduce: contiguous fp32 tensor, numel % 4 == 0, <= capacity")
        blocks = self.blocks or max(1, min(self.C.IPC_MAX_BLOCKS, (t.numel() // 4 + 1023) // 1024))
        self.C.ipc_allreduce(t.data_ptr(), t.numel(), self.data, self.sig, self.cap, self.rank, self.ctr.data_ptr(),
                             self.err.data_ptr(), blocks, torch.cuda.current_stream().cuda_stream, self.spins)
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
        for p in self._opened:
            self.C.ipc_close(p)
        for p in self._own:
            self.C.ipc_free(p)
        self._opened, self._own = [], ()
