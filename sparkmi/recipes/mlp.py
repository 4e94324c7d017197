"""Multilayer-perceptron training — distributed_multilayer_perceptron.py (R02-R07) and
pytorch_multilayer_perceptron.py (R08).

Reference flow: libsvm file -> Spark DataFrame -> dense float32 features / int64 labels ->
60/40 random_split -> DataLoader(batch 30) -> Linear(4,5)-Sigmoid-Linear(5,4)-Sigmoid-Linear(4,3)
with CE + SGD(lr 0.03) for 100 epochs -> eval (softmax/argmax, loss, accuracy).  Here the same
flow runs through sparkmi's Session reader (C++ libsvm parser), executor shards resident in HBM
and the fused whole-MLP HIP kernel (forward + CE + backward in one launch) with the fused SGD
update, captured in a HIP graph.  With no ``--data-dir`` file, the iris-shaped synthetic libsvm
text stands in for $SPARK_HOME/data/mllib/sample_multiclass_classification_data.txt.
"""
import dataclasses
import os

import torch

from ..api.session import Session
from ..data.dataset import DeviceLoader
from ..data.synthetic import iris_libsvm_text
from ..models.mlp import MultilayerPerceptron
from ..optim import SGD
from ..train.config import TrainConfig, parse
from ..train.trainer import Trainer, setup_executor
from .common import evaluate_classifier, run, shard


@dataclasses.dataclass
class MLPConfig(TrainConfig):
    """MLP classifier (distributed_multilayer_perceptron.py / pytorch_multilayer_perceptron.py)."""
    epochs: int = 100
    batch_size: int = 30
    lr: float = 0.03
    layers: str = "4,5,4,3"
    split_seed: int = 1234


def load_frames(cfg):
    spark = Session.builder.appName("sparkmi-mlp").getOrCreate()
    path = cfg.data_dir
    if path and os.path.isdir(path):
        path = os.path.join(path, "sample_multiclass_classification_data.txt")
    if path and os.path.exists(path):
        df = spark.read.format("libsvm").load(path)
        source = path
    else:
        df = spark.read.libsvm(iris_libsvm_text(150, seed=cfg.seed or 1234), text=True)
        source = "synthetic"
    train_df, test_df = df.randomSplit([0.6, 0.4], seed=cfg.split_seed)
    return train_df, test_df, source


def train_fn(cfg):
    rank, world, device = setup_executor(cfg)
    train_df, test_df, source = load_frames(cfg)
    xtr, ytr = train_df.to_torch()
    xte, yte = test_df.to_torch()
    idx = torch.from_numpy(shard(len(ytr), rank, world, cfg.seed))
    full = len(idx) % cfg.batch_size == 0
    # whole batches only: the fixed-buffer loader (each step gathers its shuffled batch inside the
    # step's HIP graph); a ragged last batch keeps the per-batch gather
    loader = DeviceLoader([xtr[idx], ytr[idx]], cfg.batch_size, device, shuffle=True, drop_last=full,
                          seed=cfg.seed + 1000 * rank, fixed=full)
    torch.manual_seed(cfg.seed)
    layers = [int(v) for v in cfg.layers.split(",")]
    model = MultilayerPerceptron(layers)
    # a ragged last batch changes the input shape: capture only when all batches are full
    if len(idx) % cfg.batch_size:
        cfg = dataclasses.replace(cfg, graph=False)
    # one executor: each step is ONE kernel (forward + CE + backward + SGD, csrc/kernels/mlp.hip)
    trainer = Trainer(model, lambda m, x, y: m.loss(x, y), lambda flat: SGD(flat, lr=cfg.lr), cfg, device, rank,
                      world, "mlp", shadow=False, fused_step=lambda m, o, x, y: m.fused_sgd_step(o, x, y),
                      fused_grad=lambda m, x, y: m.fused_grad_step(x, y),
                      fused_steps=lambda m, o, bs: m.fused_sgd_steps(o, bs))
    stats = trainer.fit(loader, cfg.epochs)
    trainer.close()
    out = dict(stats, data=source, world=world, n_train=len(ytr), n_test=len(yte))
    if rank == 0:
        model.eval()
        out.update(evaluate_classifier(model, xte.to(device), yte.to(device)))
        out["state_dict"] = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    return out if rank == 0 else None


def main(argv=None):
    cfg = parse(MLPConfig, argv)
    res = run(train_fn, cfg)
    if cfg.verbose and res is not None:
        print({k: v for k, v in res.items() if k != "state_dict"})
    return res


if __name__ == "__main__":
    main()
