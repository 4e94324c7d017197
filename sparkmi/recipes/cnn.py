"""FashionMNIST CNN training — distributed_cnn.py (R09-R14) and pytorch_cnn.py (R15).

Reference: batch 32, SGD lr 0.01, CE, 3 epochs, FashionMNISTModel(1, 10, 10)
(distributed_cnn.py:109-147).  Differences by design: every executor trains on its own disjoint
shard of the TRAIN set (the reference iterated the test loader, Q3, through a sampler fixed to
rank 0 of 2, Q2) and gradients really are averaged (Q1).  The shard is uploaded to HBM once as
uint8; each step is the batch gather (device cursor, sparkmi/data/dataset.py DeviceLoader
fixed=True) + one fused HIP kernel for forward+backward of the whole network and the SGD update
on a single executor (data-parallel: the kernel leaves the batch gradient, then the IPC
all-reduce and SGD), replayed as multi-step HIP graphs (cfg.unroll steps per launch).
"""
import dataclasses

import numpy as np
import torch

from ..data.dataset import DeviceLoader
from ..data.idx import load_fashion_mnist
from ..data.synthetic import fashion_mnist_like
from ..models.cnn import FashionMNISTModel
from ..optim import SGD
from ..train.config import TrainConfig, parse
from ..train.trainer import Trainer, setup_executor
from .common import evaluate_classifier, run, shard


@dataclasses.dataclass
class CNNConfig(TrainConfig):
    """FashionMNIST CNN (distributed_cnn.py / pytorch_cnn.py)."""
    local_mode: bool = False       # TorchDistributor(local_mode=False), distributed_cnn.py:227-230
    epochs: int = 3
    batch_size: int = 32
    lr: float = 0.01
    hidden_units: int = 10
    conv_dtype: str = "fp32"       # "bf16": convolutions on bf16 matrix cores (BASELINE's CNN config)
    n_train: int = 60000
    n_test: int = 10000


def load_data(cfg):
    real = load_fashion_mnist(cfg.data_dir) if cfg.data_dir else None
    if real is not None:
        (xtr, ytr), (xte, yte) = real
        return (torch.from_numpy(np.ascontiguousarray(xtr)), torch.from_numpy(ytr)), \
               (torch.from_numpy(np.ascontiguousarray(xte)), torch.from_numpy(yte)), "fashion-mnist"
    xtr, ytr = fashion_mnist_like(cfg.n_train, seed=cfg.seed)
    xte, yte = fashion_mnist_like(cfg.n_test, seed=cfg.seed + 1)
    return (xtr, ytr), (xte, yte), "synthetic"


def train_fn(cfg):
    rank, world, device = setup_executor(cfg)
    (xtr, ytr), (xte, yte), source = load_data(cfg)
    idx = torch.from_numpy(shard(len(ytr), rank, world, cfg.seed))
    # fixed-buffer loader: each step gathers its shuffled batch inside the step's HIP graph
    loader = DeviceLoader([xtr[idx], ytr[idx]], cfg.batch_size, device, shuffle=True, drop_last=True,
                          seed=cfg.seed + 1000 * rank, fixed=True)
    torch.manual_seed(cfg.seed)
    model = FashionMNISTModel(1, cfg.hidden_units, 10, dtype=cfg.conv_dtype)
    trainer = Trainer(model, lambda m, x, y: m.loss(x, y), lambda flat: SGD(flat, lr=cfg.lr), cfg, device, rank,
                      world, "cnn", shadow=False, fused_step=lambda m, o, x, y: m.fused_sgd_step(o, x, y),
                      fused_grad=lambda m, x, y: m.fused_grad_step(x, y))
    stats = trainer.fit(loader, cfg.epochs)
    trainer.close()
    out = dict(stats, data=source, world=world, train_samples_per_rank=len(idx))
    if rank == 0:
        model.eval()
        out.update(evaluate_classifier(model, xte.to(device), yte.to(device)))
        out["train_samples_per_s"] = stats["steps"] * cfg.batch_size * world / max(stats["time_s"], 1e-9)
        out["state_dict"] = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    return out if rank == 0 else None


def main(argv=None):
    cfg = parse(CNNConfig, argv)
    res = run(train_fn, cfg)
    if cfg.verbose and res is not None:
        print({k: v for k, v in res.items() if k != "state_dict"})
    return res


if __name__ == "__main__":
    main()
