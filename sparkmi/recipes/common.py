"""Shared recipe plumbing: executor launch (sequential in-process or Distributor), data sharding,
evaluation helpers."""
import os

import numpy as np
import torch

from ..api.distributor import Distributor


def run(train_fn, cfg):
    """world == 1: run in this process (the pytorch_*.py scripts); world > 1: one executor
    process per MI355X through Distributor (the distributed_*.py scripts' TorchDistributor)."""
    if cfg.world <= 1:
        return train_fn(cfg)
    use_gpu = cfg.device != "cpu" and torch.cuda.device_count() > 0
    # SPARKMI_SHARE_GPUS=1: several executors per device (tests on a one-GPU box; gloo backend)
    share = os.environ.get("SPARKMI_SHARE_GPUS", "0") == "1"
    return Distributor(num_processes=cfg.world, local_mode=getattr(cfg, "local_mode", True), use_gpu=use_gpu,
                       share_gpus=share,
                       max_restarts=getattr(cfg, "max_restarts", 0),
                       progress_timeout=getattr(cfg, "progress_timeout", 0.0) or None).run(train_fn, cfg)


def shard(n, rank, world, seed=0):
    """Disjoint, equal-size rank shard of range(n) after a seeded shuffle (DistributedSampler
    semantics with drop_last; fixes the reference's num_replicas=2, rank=0 sampler, Q2)."""
    perm = np.random.default_rng(seed).permutation(n)
    per = n // world
    return np.sort(perm[rank * per:(rank + 1) * per])


def accuracy_fn(y_true, y_pred):
    """Percent of equal labels (distributed_multilayer_perceptron.py:56-59)."""
    correct = torch.eq(y_true, y_pred).sum().item()
    return correct / max(1, len(y_pred)) * 100.0


@torch.no_grad()
def evaluate_classifier(logits_fn, x, y, batch_size=1024):
    """Full-test-set mean CE loss and accuracy (the reference's eval_func reports the last
    batch's accuracy only, Q18)."""
    tot_loss, correct, n = 0.0, 0, 0
    for i in range(0, len(y), batch_size):
        xb, yb = x[i:i + batch_size], y[i:i + batch_size]
        z = logits_fn(xb).float()
        tot_loss += torch.nn.functional.cross_entropy(z, yb, reduction="sum").item()
        correct += (z.argmax(1) == yb).sum().item()
        n += len(yb)
    return {"test_loss": tot_loss / max(1, n), "test_acc": 100.0 * correct / max(1, n), "n_test": n}
