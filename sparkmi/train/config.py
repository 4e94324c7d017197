"""Typed recipe configuration with CLI overrides.

The reference keeps hyper-parameters as module constants (distributed_lstm.py:60-66,
pytorch_machine_translator.py:108-117) and cluster shape in SparkConf.  Here every recipe has a
dataclass whose defaults ARE the reference's constants; ``parse(cls, argv)`` builds an argparse
parser from the fields (``--batch-size 64 --world 8 --no-graph``), and ``from_env`` honours the
Spark / torchrun variables (``spark.executor.instances`` -> world size).
"""
import argparse
import dataclasses
import json
import os
import typing


@dataclasses.dataclass
class TrainConfig:
    world: int = 1                 # executors (one per MI355X); spark.executor.instances
    epochs: int = 1
    max_steps: int = 0             # 0: run all epochs
    batch_size: int = 32
    lr: float = 1e-3
    seed: int = 0
    device: str = "auto"           # auto | cuda | cpu
    graph: bool = True             # capture the step in a HIP graph (single executor)
    ckpt_dir: str = ""             # checkpoint directory ("" disables)
    ckpt_every: int = 0            # steps between checkpoints (0: end of each epoch)
    resume: bool = True            # resume from ckpt_dir/latest when present
    metrics: str = ""              # per-rank JSONL path prefix ("" disables the file)
    log_every: int = 50
    data_dir: str = ""             # real dataset location if present (else synthetic)
    n_train: int = 0               # synthetic dataset size (0: reference size)
    n_test: int = 0
    bucket_mb: float = 64.0        # data-parallel gradient bucket size
    zero: bool = False             # ZeRO-1: reduce-scatter + sharded optimizer + all-gather
    local_mode: bool = True        # TorchDistributor local_mode (False: barrier-task cluster mode)
    progress_timeout: float = 0.0  # s without step progress on a rank -> group failure (0: off)
    max_restarts: int = 0          # group restarts from the last checkpoint after a failure
    phase_timing: bool = False     # graph steps as separate phase graphs + events (timing, slower)
    unroll: int = 16               # fixed-buffer loaders: steps per replayed multi-step graph
    sparse_embedding: bool = False  # DP: exchange the model's embedding gradient row-sparse
                                    # (models exposing ``sparse_rows()``, e.g. the LSTM)
    verbose: bool = True

    def to_json(self):
        return json.dumps(dataclasses.asdict(self))


def _arg_type(tp):
    if tp in (int, float, str):
        return tp
    origin = typing.get_origin(tp)
    if origin is typing.Union:
        args = [a for a in typing.get_args(tp) if a is not type(None)]
        return _arg_type(args[0])
    return str


def parse(cls, argv=None, **defaults):
    """Instantiate ``cls`` (a TrainConfig dataclass) from command-line arguments."""
    hints = typing.get_type_hints(cls)
    p = argparse.ArgumentParser(description=cls.__doc__)
    base = cls(**defaults)
    for f in dataclasses.fields(cls):
        name = "--" + f.name.replace("_", "-")
        cur = getattr(base, f.name)
        tp = hints[f.name]
        if tp is bool:
            p.add_argument(name, dest=f.name, action=argparse.BooleanOptionalAction, default=cur)
        else:
            p.add_argument(name, dest=f.name, type=_arg_type(tp), default=cur)
    ns = p.parse_args(argv)
    cfg = cls(**vars(ns))
    return from_env(cfg, explicit=set(k for k in vars(ns) if getattr(ns, k) != getattr(base, k)))


def from_env(cfg, explicit=()):
    """Fill ``world`` from SPARKMI_WORLD / spark.executor.instances when not given explicitly."""
    if "world" not in explicit:
        w = os.environ.get("SPARKMI_WORLD") or os.environ.get("SPARK_EXECUTOR_INSTANCES")
        if w:
            cfg.world = int(w)
    return cfg


def resolve_device(cfg):
    import torch
    if cfg.device == "auto":
        return "cuda" if torch.cuda.is_available() else "cpu"
    return cfg.device
