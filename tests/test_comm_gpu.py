"""T6 on one MI355X: the native comm layer (csrc/comm).

* IPC one-shot all-reduce with TWO processes sharing the GPU (IPC handles work across processes
  on one device): results equal the rank-ordered fp32 sum bit for bit, over
  several epochs (both staging halves) and sizes, including a bucket that does not fill a block.
* The native RCCL communicator (world 1 on one GPU — RCCL refuses two ranks on one device):
  bootstrap through the TCPStore, every collective entry point, async-error query, abort.
"""
import sys

import cloudpickle
import pytest
import torch

pytestmark = pytest.mark.gpu

cloudpickle.register_pickle_by_value(sys.modules[__name__])

SIZES = [4, 256, 7744, 65536]  # floats: MLP-sized, CNN-sized (7,740 params padded), 256 KB


def _ipc_fn():
    import torch
    from sparkmi.parallel import init_distributed, destroy
    from sparkmi.parallel.comm import IpcAllReduce
    rank, world, dev = init_distributed()
    ar = IpcAllReduce(cap_floats=1 << 16)
    out = []
    for it in range(3):
        for n in SIZES:
            g = torch.Generator().manual_seed(1000 * it + n + rank)
            x = torch.randn(n, generator=g).to(dev)
            ar(x)
            out.append(x.cpu())
    torch.cuda.synchronize()
    ar.check()
    ar.close()
    destroy()
    return out


def test_ipc_allreduce_two_processes_one_gpu():
    from sparkmi.api import Distributor
    res = Distributor(num_processes=2, use_gpu=True, share_gpus=True, env={"SPARKMI_DIST_BACKEND": "gloo"}, log_sink=None,
                      timeout=300).run(_ipc_fn)
    k = 0
    for it in range(3):
        for n in SIZES:
            a = torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + n))
            b = torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + n + 1))
            assert torch.equal(res[k], a + b), (it, n)
            k += 1


def _rccl_fn():
    import torch
    from sparkmi.parallel import init_distributed, destroy
    from sparkmi.parallel.comm import NativeComm
    rank, world, dev = init_distributed()
    c = NativeComm()
    x = torch.arange(16, dtype=torch.float32, device=dev)
    c.all_reduce(x)
    o = torch.empty(16, device=dev)
    c.all_gather(o, x)
    r = torch.empty(16, device=dev)
    c.reduce_scatter(r, x)
    c.broadcast(x, 0)
    torch.cuda.synchronize()
    e = c.async_error()
    c.abort()
    destroy()
    return x.cpu(), o.cpu(), r.cpu(), e


def test_native_rccl_world1():
    from sparkmi.api import Distributor
    x, o, r, e = Distributor(num_processes=1, use_gpu=True, log_sink=None,
                             timeout=300).run(_rccl_fn)
    ref = torch.arange(16, dtype=torch.float32)
    assert torch.equal(x, ref) and torch.equal(o, ref) and torch.equal(r, ref) and e == 0


def _mlp_dp(steps, use_dp):
    import torch
    from sparkmi.models.mlp import MultilayerPerceptron
    from sparkmi.optim import SGD
    from sparkmi.parallel import DataParallel, destroy, init_distributed
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    rank, world, dev = init_distributed()
    torch.manual_seed(0)
    model = MultilayerPerceptron((4, 5, 4, 3)).to(dev).train()
    flat = FlatParams(model, shadow=False)
    opt = SGD(flat, lr=0.1)
    ddp = DataParallel(flat) if use_dp else None
    info = {"ipc": ddp is not None and ddp.ipc is not None, "graph_safe": ddp is not None and ddp.graph_safe}
    runner = StepRunner(model, lambda m, x, y: m.loss(x, y), opt, ddp, graph=True)
    g = torch.Generator().manual_seed(5)
    X = torch.rand(steps, 60, 4, generator=g) * 2 - 1
    Y = torch.randint(0, 3, (steps, 60), generator=g)
    per = 60 // world
    for i in range(steps):
        runner.step(X[i, rank * per:(rank + 1) * per].to(dev), Y[i, rank * per:(rank + 1) * per].to(dev))
    torch.cuda.synchronize()
    out = flat.master.cpu().clone()
    if ddp is not None:
        ddp.close()
    destroy()
    return out, info


def test_ipc_data_parallel_whole_step_graph():
    """MLP data parallelism over the IPC all-reduce with the WHOLE step in one HIP graph (two
    processes sharing the GPU) == one process at twice the batch."""
    from sparkmi.api import Distributor
    dp, info = Distributor(num_processes=2, use_gpu=True, share_gpus=True, env={"SPARKMI_DIST_BACKEND": "gloo"}, log_sink=None,
                           timeout=300).run(_mlp_dp, 12, True)
    assert info["ipc"] and info["graph_safe"]
    single, _ = Distributor(num_processes=1, use_gpu=True, log_sink=None, timeout=300).run(_mlp_dp, 12, False)
    torch.testing.assert_close(dp, single, atol=1e-5, rtol=1e-5)
