"""Counter-based dropout RNG shared bit-for-bit by the HIP kernels and the torch reference path.

keep(i) = hash(seed, i) >= round(p * 2^32), seed = step_seed * 0x9E3779B9 + salt (mod 2^32).
``step_seed`` lives in a device int32 tensor that a captured kernel bumps once per step, so a
replayed HIP graph draws a fresh mask each step; ``salt`` is a static per-call-site constant
handed out at module construction.  Masks are never stored: the backward recomputes them.
Mirrors ``smi_hash``/``smi_seed`` in csrc/include/smi_common.h.
"""
import contextlib
import itertools

import torch

_M32 = 0xFFFFFFFF
_salts = itertools.count(1)


def reset_salts():
    """Restart the per-call-site salt sequence (a run's entry point: models built after this get
    the same dropout streams as in a fresh process)."""
    global _salts
    _salts = itertools.count(1)


@contextlib.contextmanager
def salt_scope(base: int = 1):
    """Modules built inside draw the salts base, base + 1, ... of a stream of their own; the
    process-wide sequence is restored afterwards.  The root models (Transformer, LSTM) build their
    submodules in one, so a model's dropout masks depend only on its own structure and ``salt_base``
    — not on how many models the process built before it (an eval model beside a training model,
    an MLlib Pipeline's stages, a test suite)."""
    global _salts
    saved = _salts
    _salts = itertools.count(int(base))
    try:
        yield
    finally:
        _salts = saved


def new_salt() -> int:
    """A fresh static per-call-site salt (deterministic construction order)."""
    return (next(_salts) * 0x2545F491) & _M32


def threshold(p: float) -> int:
    if p <= 0.0:
        return 0
    return min(int(round(p * 4294967296.0)), _M32)


def scale(p: float) -> float:
    return 1.0 / (1.0 - p) if p > 0.0 else 1.0


def mix_seed(step_seed: int, salt: int) -> int:
    return (step_seed * 0x9E3779B9 + salt) & _M32


def hash_u32(seed: int, idx: torch.Tensor) -> torch.Tensor:
    """smi_hash on an int64 tensor of element indices (values < 2^32)."""
    s = ((seed * 0x85EBCA77 + 0x165667B1) & _M32)
    h = ((idx * 0x9E3779B1) & _M32) ^ s
    h = h ^ (h >> 16)
    h = (h * 0x7FEB352D) & _M32
    h = h ^ (h >> 15)
    h = (h * 0x846CA68B) & _M32
    h = h ^ (h >> 16)
    return h


def keep_mask(shape, p: float, step_seed: int, salt: int, device=None) -> torch.Tensor:
    """Boolean keep-mask over a contiguous tensor of ``shape`` (element index = flat offset)."""
    n = 1
    for d in shape:
        n *= d
    idx = torch.arange(n, dtype=torch.int64, device=device)
    h = hash_u32(mix_seed(step_seed, salt), idx)
    return (h >= threshold(p)).reshape(shape)


class DropoutRNG(torch.nn.Module):
    """Per-model dropout step seed as a non-persistent int32 device buffer.

    ``advance()`` bumps it on the device (captured in the training-step graph on GPU), so every
    step draws fresh masks; submodules hold a reference to this module, not to the tensor, so
    ``model.to(device)`` keeps them in sync.  Not part of the state_dict (reference key parity).
    """

    def __init__(self, seed: int = 0):
        super().__init__()
        self.register_buffer("seed", torch.tensor([int(seed) & 0x7FFFFFFF], dtype=torch.int32), persistent=False)

    def advance(self):
        from .. import _native
        if _native.use_native(self.seed):
            _native.C().seed_inc(self.seed.data_ptr(), _native.stream())
        else:
            self.seed.add_(1)

    def current(self) -> int:
        return int(self.seed.item())

    def ptr(self) -> int:
        return self.seed.data_ptr()

    def reseed(self, seed: int):
        self.seed.fill_(int(seed) & 0x7FFFFFFF)
