"""The multi-cut optimizer-update plan (sparkmi/train/runner.py _EarlyUpdate) on CPU, with a mock
optimizer: which flat ranges are updated at which cut of the backward.  Side cuts hand over
everything reported final so far plus the launched parameters; the late cut (main stream) only
its launched parameters; a parameter reported again after a cut stays out of that cut's plan.
The GPU counterpart pins the arithmetic bitwise: tests/test_f32_gpu.py::test_transformer_early_update_bitwise."""
import pytest
import torch

from sparkmi.ops import _grad
from sparkmi.train import runner as R
from sparkmi.utils.flat import FlatParams


class _Opt:
    def __init__(self, flat):
        self.flat = flat
        self.calls = []

    def step_ranges(self, rs):
        self.calls.append(list(rs))


def _setup():
    m = torch.nn.Sequential(*[torch.nn.Linear(8, 8, bias=False) for _ in range(5)])
    flat = FlatParams(m, device="cpu", shadow=False)
    return flat, list(flat.params), _Opt(flat)


def _range(flat, i):
    o = flat.offsets[i]
    return (o, o + (flat.params[i].numel() + 63) // 64 * 64)


def test_plans_per_cut_and_late_cut(monkeypatch):
    monkeypatch.setattr(R, "EARLY_UPDATE_CUTS", 2)
    monkeypatch.setattr(R, "LATE_UPDATE", True)
    flat, ps, opt = _setup()
    eu = R._EarlyUpdate(opt)
    # the launched parameters' reports after their cut are confirmations (CONFIRMING in _grad)
    _grad.CONFIRMING[0] = False
    eu.begin()
    eu.on_ready(ps[0])
    eu.at_cut([ps[1]])
    eu.at_cut([ps[2]])
    eu.at_cut([ps[3]])
    eu.at_cut([ps[4]], late=True)
    _grad.CONFIRMING[0] = True
    for i in (1, 2, 3, 4):
        eu.on_ready(ps[i])
    _grad.CONFIRMING[0] = False
    eu.end()
    assert opt.calls == []  # the first backward only learns
    rs = [r for r, _ in eu.plans]
    # cut 0: param 0 (ready before) + 1 (launched); cut 1: param 2; cut 2 (third side cut) not updated
    # early (EARLY_UPDATE_CUTS = 2); the late cut: param 4 only (param 3, launched on the side
    # stream, is not final on the main stream)
    assert rs[0] == [(_range(flat, 0)[0], _range(flat, 1)[1])]
    assert rs[1] == [_range(flat, 2)]
    assert rs[2] == []
    assert rs[3] == [_range(flat, 4)]
    # the next backward executes them at their cuts
    eu.begin()
    eu.on_ready(ps[0])
    eu.at_cut([ps[1]])
    eu.at_cut([ps[2]])
    eu.at_cut([ps[3]])
    eu.at_cut([ps[4]], late=True)
    eu.end()
    assert eu.used == [0, 1, 3]
    assert opt.calls == [rs[0], rs[1], rs[3]]


def test_param_reported_after_cut_is_excluded(monkeypatch):
    monkeypatch.setattr(R, "EARLY_UPDATE_CUTS", 2)
    flat, ps, opt = _setup()
    eu = R._EarlyUpdate(opt)
    _grad.CONFIRMING[0] = False
    eu.begin()
    eu.on_ready(ps[0])
    eu.on_ready(ps[1])
    eu.at_cut([])
    eu.on_ready(ps[1])  # param 1 receives more gradient after the cut (e.g. a reused module)
    eu.end()
    assert [r for r, _ in eu.plans][0] == [_range(flat, 0)]
    # a later backward in which a planned parameter shows up after its cut fails loudly
    eu.begin()
    eu.on_ready(ps[0])
    eu.on_ready(ps[1])
    eu.at_cut([])
    eu.on_ready(ps[0])
    with pytest.raises(RuntimeError):
        eu.end()
