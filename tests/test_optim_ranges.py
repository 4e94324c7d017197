"""Adam in two parts (sparkmi/optim/adam.py step_ranges + step): element for element the
one-launch update — CPU torch path here; the HIP path is pinned bitwise in
tests/test_f32_gpu.py::test_transformer_early_update_bitwise."""
import copy

import torch

from sparkmi.optim import Adam
from sparkmi.utils.flat import FlatParams


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(17, 33), torch.nn.ReLU(), torch.nn.Linear(33, 5))


def test_adam_step_ranges_equals_one_update():
    base = _model()
    runs = []
    for split in (False, True):
        m = copy.deepcopy(base)
        flat = FlatParams(m, shadow=False)
        opt = Adam(flat, lr=1e-2, weight_decay=0.01)
        g = torch.Generator().manual_seed(1)
        for step in range(3):
            flat.grad.copy_(torch.randn(flat.numel, generator=g))
            if split:
                o = flat.offsets
                opt.step_ranges([(o[0], o[1]), (o[2], o[3])])  # two of the four parameters first
                assert opt._early
            opt.step()
            assert not opt._early
        runs.append((flat.master.clone(), opt.m.clone(), opt.v.clone(), opt.step_t.clone(), flat.grad.clone()))
    for a, b in zip(*runs):
        assert torch.equal(a, b)
    assert float(runs[1][3]) == 3.0


def test_adam_all_early_still_advances():
    m = _model()
    flat = FlatParams(m, shadow=False)
    opt = Adam(flat, lr=1e-2)
    flat.grad.normal_()
    opt.step_ranges([(0, flat.numel)])
    opt.step()
    assert float(opt.step_t) == 1.0
    assert torch.count_nonzero(flat.grad) == 0


def test_adam_step_ranges_sharded_equals_one_update():
    """ZeRO-1 (compact moments over owned pieces): updating parts of the pieces early (the per-bucket
    update of sparkmi/parallel/ddp.py) then step() == the one multi-range update; a range outside
    the owned pieces is refused."""
    base = _model()
    runs = []
    for split in (False, True):
        m = copy.deepcopy(base)
        flat = FlatParams(m, shadow=False)
        n = flat.numel
        opt = Adam(flat, lr=1e-2).shard([(64, n // 2), (n // 2 + 64, n)])
        g = torch.Generator().manual_seed(2)
        for step in range(3):
            flat.grad.copy_(torch.randn(n, generator=g))
            if split:
                opt.step_ranges([(64, 128), (n // 2 + 64, n)])  # part of piece 0, all of piece 1
            opt.step()
            assert not opt._early
        runs.append((flat.master.clone(), opt.m.clone(), opt.v.clone(), opt.step_t.clone()))
    for a, b in zip(*runs):
        assert torch.equal(a, b)
    import pytest
    with pytest.raises(ValueError):
        opt.step_ranges([(0, 64)])
