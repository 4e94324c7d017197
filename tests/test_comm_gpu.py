"""T6 on one MI355X: the native comm layer (csrc/comm/ipc_allreduce.hip).

* IPC one-shot AND two-shot all-reduce with 2, 4 and 8 processes sharing the GPU (IPC handles work
  across processes on one device): results equal the rank-ordered fp32 sum bit
  for bit, over several epochs (both staging halves), both kernels interleaved on one signal
  array, and sizes from 16 B to 16 MB (ragged chunks, buckets that do not fill a block).
* Zero-copy two-shot (algo 3: peers read each other's IPC-registered buffer in place, no staging)
  at 2, 4 and 8 processes: bit-identical rank-order sums at every size and at a non-zero offset,
  interleaved with the staged kernels on one signal array, and every rank overwrites its buffer
  right after each call with no host sync (the third signal round must keep that write behind
  every peer's reads).
* Peer loss: rank 1 skips one all-reduce -> rank 0's kernel times out within the configured
  bound, its bucket is NaN (never a finite partial sum) and check() raises IpcPeerLost.
"""
import sys

import cloudpickle
import pytest
import torch

pytestmark = pytest.mark.gpu

cloudpickle.register_pickle_by_value(sys.modules[__name__])

# floats: MLP-sized, CNN-sized (7,740 params padded), 256 KB, a ragged 1.2 MB, LSTM-sized 12.3 MB
SIZES = [4, 256, 7744, 65536, 300004, 3075008]
CAP = 1 << 22


def _ipc_fn():
    import torch
    from sparkmi.parallel import init_distributed, destroy
    from sparkmi.parallel.comm import IpcAllReduce
    rank, world, dev = init_distributed()
    ar = IpcAllReduce(cap_floats=CAP)
    out = []
    for it in range(3):
        for n in SIZES:
            for algo in (1, 2):
                g = torch.Generator().manual_seed(1000 * it + n + rank)
                x = torch.randn(n, generator=g).to(dev)
                ar(x, algo=algo)
                out.append(x.cpu())
    torch.cuda.synchronize()
    ar.check()
    ar.close()
    destroy()
    return out


@pytest.mark.timeout(400)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_ipc_allreduce_processes_one_gpu(world):
    """2, 4 and 8 ranks sharing the GPU: the 8-rank signal slots, the 4- and 8-chunk two-shot
    ranges (ragged last chunks) and the rank-order sums the node's 8-GPU run relies on."""
    from sparkmi.api import Distributor
    res = Distributor(num_processes=world, use_gpu=True, share_gpus=True, env={"SPARKMI_DIST_BACKEND": "gloo"},
                      log_sink=None, timeout=380).run(_ipc_fn)
    k = 0
    for it in range(3):
        for n in SIZES:
            want = torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + n))
            for r in range(1, world):  # rank order, as the kernels sum
                want = want + torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + n + r))
            for algo in (1, 2):
                assert torch.equal(res[k], want), (world, it, n, algo)
                k += 1


def _zc_fn():
    import torch
    from sparkmi.parallel import init_distributed, destroy
    from sparkmi.parallel.comm import IpcAllReduce
    rank, world, dev = init_distributed()
    ar = IpcAllReduce(cap_floats=CAP)
    buf = torch.zeros(max(SIZES) + 64, device=dev)
    assert ar.register(buf)
    out, staged = [], []
    for it in range(3):
        for n in SIZES:
            off = 64 if (it + n) % 2 else 0  # a non-zero (16-B aligned) offset too
            g = torch.Generator().manual_seed(1000 * it + n + rank)
            buf[off:off + n].copy_(torch.randn(n, generator=g).to(dev))
            ar(buf[off:off + n], algo=3)
            out.append(buf[off:off + n].clone())  # device copy: no host sync before the next overwrite
            y = torch.full((256,), float(rank), device=dev)
            ar(y, algo=1 + (n % 2))  # a staged call on the same signal array between zero-copy ones
            staged.append(y)
            buf.fill_(-1.0)  # the next backward's writes, right behind the call
    torch.cuda.synchronize()
    ar.check()
    ar.close()
    destroy()
    return [t.cpu() for t in out], [float(t[0]) for t in staged]


@pytest.mark.timeout(400)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_ipc_zero_copy_allreduce_processes_one_gpu(world):
    """the zero-copy two-shot gives the exact rank-order sums of the staged kernels,
    at 2, 4 and 8 ranks, with each rank's buffer overwritten immediately after every call."""
    from sparkmi.api import Distributor
    res, staged = Distributor(num_processes=world, use_gpu=True, share_gpus=True,
                              env={"SPARKMI_DIST_BACKEND": "gloo"}, log_sink=None, timeout=380).run(_zc_fn)
    k = 0
    for it in range(3):
        for n in SIZES:
            want = torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + n))
            for r in range(1, world):
                want = want + torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + n + r))
            assert torch.equal(res[k], want), (world, it, n)
            k += 1
    assert staged == [float(world * (world - 1) // 2)] * len(staged)


def _lost_fn(lost_algo=2):
    import time
    import torch
    from sparkmi.parallel import init_distributed, destroy
    from sparkmi.parallel.comm import IpcAllReduce, IpcPeerLost
    rank, world, dev = init_distributed()
    ar = IpcAllReduce(cap_floats=1 << 16, timeout_s=1.0)
    reg = torch.zeros(1 << 17, device=dev)
    if lost_algo == 3:
        assert ar.register(reg)

    def ones(n):  # the tensor a call reduces (algo 3: a slice of the registered buffer)
        if lost_algo == 3:
            return reg[:n].fill_(1.0)
        return torch.ones(n, device=dev)
    res = {}
    for algo in (1, 2) + ((3,) if lost_algo == 3 else ()):
        x = ones(4096) if algo == 3 else torch.ones(4096, device=dev)
        ar(x, algo=algo)  # healthy call
        torch.cuda.synchronize()
        res[f"ok{algo}"] = float(x[0])
    dist_barrier = torch.distributed.barrier
    dist_barrier()  # every peer finished its healthy calls before rank 0 goes alone
    if rank == 0:
        x = ones(65536)
        t0 = time.time()
        ar(x, algo=lost_algo)  # rank 1 never joins this one
        torch.cuda.synchronize()
        res["wait_s"] = time.time() - t0
        res["finite"] = int(torch.isfinite(x).sum())
        try:
            ar.check()
            res["raised"] = False
        except IpcPeerLost:
            res["raised"] = True
        # once a loss is recorded (sticky), a later call poisons at once, no polling
        y = ones(65536)
        t0 = time.time()
        ar(y, algo=lost_algo)
        torch.cuda.synchronize()
        res["wait2_s"] = time.time() - t0
        res["finite2"] = int(torch.isfinite(y).sum())
    allr = [None] * world
    torch.distributed.all_gather_object(allr, res)  # Distributor.run returns rank 0's value
    destroy()
    return allr


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,lost_algo", [(2, 2), (4, 2), (2, 3), (4, 3)])
def test_ipc_peer_lost_poisons_and_raises(world, lost_algo):
    from sparkmi.api import Distributor
    res = Distributor(num_processes=world, use_gpu=True, share_gpus=True, env={"SPARKMI_DIST_BACKEND": "gloo"},
                      log_sink=None, timeout=280).run(_lost_fn, lost_algo)
    r0, r1 = res[0], res[1]
    assert r0["ok1"] == r0["ok2"] == r1["ok1"] == r1["ok2"] == float(world)
    if lost_algo == 3:
        assert r0["ok3"] == r1["ok3"] == float(world)
    assert r0["raised"] and r0["finite"] == 0, r0  # poisoned, loud
    assert r0["wait_s"] < 30.0, r0  # bounded by the configured timeout (1 s of polling)
    assert r0["finite2"] == 0 and r0["wait2_s"] < 0.5, r0  # poisoned without another timeout
