"""Executor-side data path: partitioning, samplers and HBM-resident / streamed loaders.

Replaces the reference's DataLoader + DistributedSampler + random_split stack
(distributed_multilayer_perceptron.py:82-94, distributed_cnn.py:109-124,
distributed_lstm.py:147-153) and fixes its sharding bugs: every executor gets
a disjoint shard chosen by its real rank.

MI355X design: each executor's whole partition is uploaded ONCE into HBM
(288 GB holds every reference dataset many times over); per epoch a device-side permutation is
drawn and each minibatch is a gather from HBM (HIP gather kernel, fused with uint8 -> float
``ToTensor`` scaling for images).  For data larger than HBM, :class:`PinnedStreamLoader`
double-buffers pinned host batches onto the device on a side HIP stream.
"""
import math

import numpy as np
import torch

from .. import _native


class ArrayDataset:
    """TensorDataset equivalent (indexable tuple of equally long tensors/arrays)."""

    def __init__(self, *arrays):
        n = len(arrays[0])
        assert all(len(a) == n for a in arrays), "all arrays must have the same length"
        self.arrays = [a if isinstance(a, torch.Tensor) else torch.as_tensor(np.asarray(a)) for a in arrays]

    def __len__(self):
        return len(self.arrays[0])

    def __getitem__(self, i):
        return tuple(a[i] for a in self.arrays)

    def subset(self, idx):
        idx = torch.as_tensor(idx, dtype=torch.long)
        return ArrayDataset(*[a[idx] for a in self.arrays])


def random_split(dataset, lengths, seed=None):
    """torch.utils.data.random_split semantics (fractions or absolute lengths), seeded (Q19)."""
    n = len(dataset)
    if all(isinstance(x, float) for x in lengths) and abs(sum(lengths) - 1.0) < 1e-6:
        sizes = [int(math.floor(n * f)) for f in lengths]
        for i in range(n - sum(sizes)):
            sizes[i % len(sizes)] += 1
    else:
        sizes = list(lengths)
    if sum(sizes) != n:
        raise ValueError("sum of lengths must equal dataset length")
    g = torch.Generator()
    g.manual_seed(0 if seed is None else int(seed))
    perm = torch.randperm(n, generator=g)
    out, off = [], 0
    for s in sizes:
        out.append(dataset.subset(perm[off:off + s]))
        off += s
    return out


class DistributedSampler:
    """Correct rank partitioning (fixes Q2's hard-coded num_replicas=2, rank=0): indices of
    rank r are perm[r::world] of a (seed+epoch)-shuffled, padded-to-divisible index list —
    torch.utils.data.DistributedSampler semantics (torch/utils/data/distributed.py:134)."""

    def __init__(self, n, num_replicas=None, rank=None, shuffle=True, seed=0, drop_last=False):
        from ..parallel import rank as _rank, world_size as _ws
        self.n = n if isinstance(n, int) else len(n)
        self.num_replicas = num_replicas if num_replicas is not None else _ws()
        self.rank = rank if rank is not None else _rank()
        if not 0 <= self.rank < self.num_replicas:
            raise ValueError(f"rank {self.rank} out of range for {self.num_replicas} replicas")
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0
        if drop_last and self.n % self.num_replicas:
            self.num_samples = self.n // self.num_replicas
        else:
            self.num_samples = math.ceil(self.n / self.num_replicas)
        self.total_size = self.num_samples * self.num_replicas

    def set_epoch(self, epoch):
        self.epoch = epoch

    def indices(self):
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        if not self.drop_last:
            pad = self.total_size - len(idx)
            if pad > 0:
                idx += (idx * math.ceil(pad / max(1, len(idx))))[:pad]
        else:
            idx = idx[:self.total_size]
        return idx[self.rank:self.total_size:self.num_replicas]

    def __iter__(self):
        return iter(self.indices())

    def __len__(self):
        return self.num_samples


def gather_rows(src: torch.Tensor, idx: torch.Tensor, out=None, scale=None, out_dtype=None):
    """out[i] = src[idx[i]] (rows of any width); on GPU a HIP gather kernel with 16-B
    vectorised row copies, optionally fused with uint8 -> float scaling (ToTensor's /255)."""
    if src.is_cuda and _native.use_native(src):
        idx = idx.to(device=src.device, dtype=torch.int64).contiguous()
        src = src.contiguous()
        shape = (idx.shape[0],) + tuple(src.shape[1:])
        row = int(np.prod(src.shape[1:])) if src.dim() > 1 else 1
        C = _native.C()
        if scale is not None and src.dtype == torch.uint8:
            dt = out_dtype or torch.float32
            out = out if out is not None else torch.empty(shape, device=src.device, dtype=dt)
            C.gather_u8_scale(src.data_ptr(), idx.data_ptr(), out.data_ptr(), idx.shape[0], row, float(scale),
                              int(dt == torch.bfloat16), _native.stream())
            return out
        out = out if out is not None else torch.empty(shape, device=src.device, dtype=src.dtype)
        C.gather_rows(src.data_ptr(), idx.data_ptr(), out.data_ptr(), idx.shape[0], row * src.element_size(),
                      _native.stream())
        return out
    res = src[idx.to(src.device)]
    if scale is not None:
        res = res.to(out_dtype or torch.float32) * scale
    return res


class DeviceLoader:
    """HBM-resident minibatch loader for one executor's shard.

    ``arrays`` are uploaded once to ``device``; each epoch draws a device-side permutation
    (seeded by seed+epoch: reproducible, identical on every run) and yields gathered batches.
    ``image_scale`` applies the uint8 -> float ``/255`` of torchvision's ToTensor inside the
    gather (first tensor only).

    ``fixed=True`` (GPU, drop_last, no image_scale): every batch lands in the SAME static buffers,
    gathered by ONE kernel that reads the epoch's permutation at a device-side cursor and advances
    it (csrc/kernels/gather.hip gather_batch).  ``pre_step()`` launches that gather; a training
    loop that installs it into its step (Trainer -> StepRunner.pre_step, ``deferred = True``) gets
    the gather captured inside the step's HIP graph — a replayed graph, or a multi-step graph of
    several steps, draws its own shuffled batches with no host work per step.  Without a consumer
    (``deferred`` False) iteration gathers eagerly, so the yielded tensors always hold the batch."""

    def __init__(self, arrays, batch_size, device, shuffle=True, drop_last=False, seed=0, image_scale=None,
                 image_dtype=torch.float32, fixed=False):
        self.device = torch.device(device)
        self.arrays = [torch.as_tensor(a).to(self.device) for a in arrays]
        self.n = len(self.arrays[0])
        self.batch_size, self.shuffle, self.drop_last, self.seed = batch_size, shuffle, drop_last, seed
        self.image_scale, self.image_dtype = image_scale, image_dtype
        self.epoch = 0
        self.skip = 0  # batches of the current epoch already consumed (exact resume)
        self.fixed = bool(fixed and drop_last and image_scale is None and self.device.type == "cuda"
                          and len(self.arrays) <= 4 and _native.use_native(self.arrays[0]))
        self.deferred = False
        if self.fixed:
            B = batch_size
            self.static = [torch.empty((B,) + tuple(a.shape[1:]), dtype=a.dtype, device=self.device)
                           for a in self.arrays]
            self._perm_buf = torch.empty(self.n, dtype=torch.int64, device=self.device)
            self._cursor = torch.zeros(1, dtype=torch.int32, device=self.device)
            self._done = torch.zeros(1, dtype=torch.int32, device=self.device)
            self._row_bytes = [a[0].numel() * a.element_size() for a in self.arrays]

    def pre_step(self):
        """Gather the next batch (device cursor) into the static buffers: one launch, graph-safe."""
        _native.C().gather_batch([a.data_ptr() for a in self.arrays], [t.data_ptr() for t in self.static],
                                 self._row_bytes, self._perm_buf.data_ptr(), self._cursor.data_ptr(),
                                 self._done.data_ptr(), self.batch_size, _native.stream())

    def set_epoch(self, e):
        self.epoch = e

    def __len__(self):
        return self.n // self.batch_size if self.drop_last else math.ceil(self.n / self.batch_size)

    def _perm(self):
        if not self.shuffle:
            return torch.arange(self.n, device=self.device)
        g = torch.Generator(device=self.device)
        g.manual_seed(self.seed + self.epoch)
        return torch.randperm(self.n, generator=g, device=self.device)

    def __iter__(self):
        perm = self._perm()
        start, self.skip = self.skip, 0
        if self.fixed:
            # stream-ordered before every gather of the epoch (eager or replayed)
            self._perm_buf.copy_(perm)
            self._cursor.fill_(start)
            for b in range(start, len(self)):
                if not self.deferred:
                    self.pre_step()
                yield tuple(self.static)
            self.epoch += 1
            return
        for b in range(start, len(self)):
            idx = perm[b * self.batch_size:(b + 1) * self.batch_size]
            out = []
            for i, a in enumerate(self.arrays):
                if i == 0 and self.image_scale is not None:
                    out.append(gather_rows(a, idx, scale=self.image_scale, out_dtype=self.image_dtype))
                else:
                    out.append(gather_rows(a, idx))
            yield tuple(out)
        self.epoch += 1


class PinnedStreamLoader:
    """Streams host minibatches to the GPU for datasets that do not fit in HBM (SURVEY §5.8 item 6,
    §2.3 pinned_ring): the native ring (csrc/io/pinned_ring.cpp, ``sparkmi._io``) owns
    ``nslots`` page-locked host slots; each batch's rows are gathered into a slot by C++ threads
    (GIL released), shipped to a ring of device buffers with hipMemcpyAsync on a dedicated copy
    stream, and guarded by HIP events: the compute stream waits on the slot's event (no host
    sync), a slot is refilled only after its previous copy landed, and a device buffer only
    after the compute that used it was queued past.  Batch i+1 is gathered and copied while
    batch i computes.  CPU: plain gathers."""

    def __init__(self, arrays, batch_size, device, shuffle=False, drop_last=True, seed=0, nslots=3, threads=4):
        self.arrays = [np.ascontiguousarray(a.numpy() if torch.is_tensor(a) else np.asarray(a)) for a in arrays]
        self.n = len(self.arrays[0])
        self.batch_size, self.shuffle, self.drop_last, self.seed = batch_size, shuffle, drop_last, seed
        self.device = torch.device(device)
        self.epoch = 0
        self.ring = None
        if self.device.type == "cuda":
            from .. import _native
            if nslots < 3:  # batch b+1 is issued before batch b is handed out: 3 slots in flight
                raise ValueError("PinnedStreamLoader needs nslots >= 3")
            self.row_bytes = [a.itemsize * int(np.prod(a.shape[1:], dtype=np.int64)) for a in self.arrays]
            self.offs, off = [], 0
            for rb in self.row_bytes:
                self.offs.append(off)
                off += (rb * batch_size + 255) // 256 * 256
            dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
            self.ring = _native.io().PinnedRing(off, nslots, dev, threads)
            self.nslots = nslots
            tdt = [torch.from_numpy(a[:1]).dtype for a in self.arrays]
            self.dev_bufs = [[torch.empty((batch_size,) + a.shape[1:], dtype=t, device=self.device)
                              for a, t in zip(self.arrays, tdt)] for _ in range(nslots)]
            self.released = [None] * nslots  # compute-stream events: the slot's device buffers are free
            self._last = None                # slot handed out most recently

    def __len__(self):
        return self.n // self.batch_size if self.drop_last else math.ceil(self.n / self.batch_size)

    def _order(self):
        return (np.random.default_rng(self.seed + self.epoch).permutation(self.n) if self.shuffle
                else np.arange(self.n)).astype(np.int64)

    def _issue(self, s, idx):
        """Gather batch rows into slot s and queue its H2D copies; returns the device views."""
        r = self.ring
        r.acquire(s)  # the previous copy out of this host slot has landed
        k = len(idx)
        rel = self.released[s]
        outs = []
        for a, rb, off, buf in zip(self.arrays, self.row_bytes, self.offs, self.dev_bufs[s]):
            r.gather(s, off, a.ctypes.data, rb, idx.ctypes.data, k)
            r.copy_async(s, off, rb * k, buf.data_ptr(), rel.cuda_event if rel is not None else 0)
            outs.append(buf[:k])
        r.commit(s)
        return outs

    def __iter__(self):
        order = self._order()
        nb = len(self)
        if self.ring is not None:
            self._release_last()
        if self.ring is None:
            for b in range(nb):
                idx = order[b * self.batch_size:(b + 1) * self.batch_size]
                yield tuple(torch.from_numpy(a[idx]) for a in self.arrays)
            self.epoch += 1
            return
        pending = None  # (slot, device views) issued but not yet handed out
        for b in range(nb):
            idx = np.ascontiguousarray(order[b * self.batch_size:(b + 1) * self.batch_size])
            s = b % self.nslots
            views = self._issue(s, idx)
            if pending is not None:
                yield self._hand_out(*pending)
            pending = (s, views)
        if pending is not None:
            yield self._hand_out(*pending)
        self.epoch += 1

    def _release_last(self):
        """The consumer asked for another batch, so everything it does with the previous one is
        queued on the compute stream: an event there frees that slot's device buffers."""
        if self._last is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self.released[self._last] = ev
            self._last = None

    def _hand_out(self, s, views):
        self._release_last()
        self.ring.wait(s, torch.cuda.current_stream(self.device).cuda_stream)  # no host sync
        self._last = s
        return tuple(views)
