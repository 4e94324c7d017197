"""Process-group bootstrap for executors (one process per MI355X).

Reads the torchrun / TorchDistributor env contract (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR,
MASTER_PORT) and initialises torch.distributed with RCCL ("nccl" on ROCm) when the
process owns a GPU, gloo otherwise.  Replaces the reference's dist.init_process_group('gloo')
(distributed_cnn.py:152 etc.) — with RCCL gradients move over xGMI instead of TCP.
"""
import datetime
import os

import torch
import torch.distributed as dist


def is_dist():
    return dist.is_available() and dist.is_initialized()


def rank():
    return dist.get_rank() if is_dist() else int(os.environ.get("RANK", 0))


def world_size():
    return dist.get_world_size() if is_dist() else int(os.environ.get("WORLD_SIZE", 1))


def local_rank():
    return int(os.environ.get("LOCAL_RANK", 0))


def init_distributed(backend=None, timeout_s=600):
    """Initialise the default process group from env vars; returns (rank, world, device)."""
    ws = int(os.environ.get("WORLD_SIZE", 1))
    use_gpu = torch.cuda.is_available() and os.environ.get("SPARKMI_FORCE_CPU", "0") != "1"
    backend = backend or os.environ.get("SPARKMI_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    if use_gpu:
        lr, ndev = local_rank(), max(1, torch.cuda.device_count())
        if lr >= ndev and ws > 1 and backend == "nccl":
            # RCCL needs one device per rank (several ranks per GPU only over gloo, in tests)
            raise RuntimeError(f"LOCAL_RANK {lr} but only {ndev} visible GPU(s): RCCL runs one executor per "
                               f"MI355X (launch at most {ndev} ranks per node, or use the gloo backend to "
                               f"share devices in tests)")
        torch.cuda.set_device(lr % ndev)
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    if ws > 1 and not is_dist():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return rank(), world_size(), device


def barrier():
    if is_dist():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def destroy():
    if is_dist():
        dist.destroy_process_group()
