"""Training checkpoint / resume (SURVEY §5.4 (b),(c); the reference saves nothing).

A checkpoint is a directory:
  model.safetensors   model.state_dict() under the reference's key names (transformer.py,
                      distributed_lstm.py ... module names), so a reference-trained state_dict
                      and ours are interchangeable;
  optim.safetensors   the optimizer's state (flat Adam m/v, lr, step; SGD momentum ...);
  rng.safetensors     torch CPU / HIP generator states;
  meta.json           step, epoch, data cursor, dropout step seeds, world size, user extras.
Rank 0 writes into a temporary sibling directory and atomically renames it into place, then
atomically rewrites ``<dir>/latest``; a crash mid-write never corrupts the last good checkpoint.
Loading uses only non-executing loaders (safetensors + JSON).
"""
import json
import os
import shutil

import torch
from safetensors.torch import load_file, save_file

from ..ops.rng import DropoutRNG


def _tensors(d, prefix=""):
    out = {}
    for k, v in d.items():
        key = f"{prefix}{k}"
        if torch.is_tensor(v):
            out[key] = v.detach().to("cpu").contiguous().clone()
        elif isinstance(v, dict):
            out.update(_tensors(v, key + "."))
        elif isinstance(v, (int, float, bool)):
            out[key] = torch.tensor(v)
        elif v is None:
            continue
        else:
            raise TypeError(f"checkpoint: cannot store {key} of type {type(v).__name__}")
    return out


def _untensors(flat):
    out = {}
    for k, v in flat.items():
        parts = k.split(".")
        d = out
        for p in parts[:-1]:
            d = d.setdefault(p, {})
        d[parts[-1]] = v
    return out


def _dropout_seeds(model):
    if model is None:
        return {}
    return {name: int(m.seed.item()) for name, m in model.named_modules() if isinstance(m, DropoutRNG)}


def _fsync_dir(path):
    try:
        fd = os.open(path, os.O_RDONLY)
        os.fsync(fd)
        os.close(fd)
    except OSError:
        pass


def save_checkpoint(path, model=None, optimizer=None, step=0, epoch=0, cursor=0, extra=None):
    """Write a checkpoint directory at ``path`` atomically (call on rank 0 only)."""
    path = os.path.abspath(path)
    parent = os.path.dirname(path)
    os.makedirs(parent, exist_ok=True)
    tmp = f"{path}.tmp-{os.getpid()}"
    if os.path.exists(tmp):
        shutil.rmtree(tmp)
    os.makedirs(tmp)
    if model is not None:
        save_file(_tensors(model.state_dict()), os.path.join(tmp, "model.safetensors"))
    if optimizer is not None:
        save_file(_tensors(optimizer.state_dict()), os.path.join(tmp, "optim.safetensors"))
    rng = {"torch_cpu": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        for i in range(torch.cuda.device_count()):
            rng[f"torch_cuda_{i}"] = torch.cuda.get_rng_state(i)
    save_file(rng, os.path.join(tmp, "rng.safetensors"))
    meta = {"step": int(step), "epoch": int(epoch), "cursor": int(cursor), "dropout_seeds": _dropout_seeds(model),
            "world_size": int(os.environ.get("WORLD_SIZE", 1)), "format": "sparkmi-ckpt-1", "extra": extra or {}}
    with open(os.path.join(tmp, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
        f.flush()
        os.fsync(f.fileno())
    _fsync_dir(tmp)
    old = None
    if os.path.exists(path):
        old = f"{path}.old-{os.getpid()}"
        os.replace(path, old)
    os.replace(tmp, path)
    _fsync_dir(parent)
    if old:
        shutil.rmtree(old, ignore_errors=True)
    return path


def load_checkpoint(path, model=None, optimizer=None, map_location="cpu", strict=True, restore_rng=True):
    """Restore model / optimizer / RNG state from a checkpoint directory; returns its meta dict."""
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    if model is not None:
        sd = load_file(os.path.join(path, "model.safetensors"), device="cpu")
        own = model.state_dict()
        sd = {k: v.to(dtype=own[k].dtype) if k in own else v for k, v in sd.items()}
        model.load_state_dict(sd, strict=strict)
        seeds = meta.get("dropout_seeds", {})
        for name, m in model.named_modules():
            if isinstance(m, DropoutRNG) and name in seeds:
                m.reseed(seeds[name])
        flat = getattr(model, "_smi_flat", None)
        if flat is not None:
            flat.refresh_shadow()
    if optimizer is not None and os.path.exists(os.path.join(path, "optim.safetensors")):
        osd = _untensors(load_file(os.path.join(path, "optim.safetensors"), device="cpu"))
        optimizer.load_state_dict(osd)
    if restore_rng:
        rng = load_file(os.path.join(path, "rng.safetensors"), device="cpu")
        torch.set_rng_state(rng["torch_cpu"])
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            for i in range(torch.cuda.device_count()):
                if f"torch_cuda_{i}" in rng:
                    torch.cuda.set_rng_state(rng[f"torch_cuda_{i}"], i)
    return meta


class CheckpointManager:
    """``<dir>/step_<N>`` checkpoints, a ``latest`` pointer, and retention of the newest ``keep``."""

    def __init__(self, directory, keep=2, rank=0):
        self.dir = os.path.abspath(directory)
        self.keep = keep
        self.rank = rank
        os.makedirs(self.dir, exist_ok=True)

    def save(self, step, model=None, optimizer=None, epoch=0, cursor=0, extra=None):
        if self.rank != 0:
            return None
        name = f"step_{int(step):09d}"
        save_checkpoint(os.path.join(self.dir, name), model, optimizer, step, epoch, cursor, extra)
        tmp = os.path.join(self.dir, f"latest.tmp-{os.getpid()}")
        with open(tmp, "w") as f:
            f.write(name)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, os.path.join(self.dir, "latest"))
        self._prune()
        return os.path.join(self.dir, name)

    def _prune(self):
        ck = sorted(d for d in os.listdir(self.dir) if d.startswith("step_") and "." not in d)
        for d in ck[:-self.keep] if self.keep > 0 else []:
            shutil.rmtree(os.path.join(self.dir, d), ignore_errors=True)

    def latest(self):
        p = os.path.join(self.dir, "latest")
        if not os.path.exists(p):
            return None
        with open(p) as f:
            name = f.read().strip()
        full = os.path.join(self.dir, name)
        return full if os.path.isdir(full) else None

    def restore(self, model=None, optimizer=None, **kw):
        p = self.latest()
        if p is None:
            return None
        return load_checkpoint(p, model, optimizer, **kw)
