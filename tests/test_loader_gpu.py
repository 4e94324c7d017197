"""Graph-resident batch gather (DeviceLoader(fixed=True), csrc/kernels/gather.hip gather_batch) and
the Trainer's bound / multi-step replay of it (the recipe path runs like the
benchmark's step)."""
import dataclasses

import pytest
import torch

dev = "cuda"


@pytest.mark.gpu
def test_gather_batch_device_cursor_matches_index_gather():
    from sparkmi.data.dataset import DeviceLoader
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 256, (203, 28, 28), generator=g, dtype=torch.uint8)
    y = torch.randint(0, 10, (203,), generator=g)
    a = DeviceLoader([x, y], 16, dev, shuffle=True, drop_last=True, seed=5)
    b = DeviceLoader([x, y], 16, dev, shuffle=True, drop_last=True, seed=5, fixed=True)
    assert b.fixed and not a.fixed
    for epoch in range(2):
        got = [tuple(t.clone() for t in bt) for bt in b]
        ref = list(a)
        assert len(got) == len(ref) == 203 // 16
        for (gx, gy), (rx, ry) in zip(got, ref):
            assert torch.equal(gx, rx) and torch.equal(gy, ry)
    # the cursor advanced on the device once per batch
    assert int(b._cursor.item()) == 203 // 16


def _trainer(fixed, steps, unroll, world=1, index=True):
    from sparkmi.data.dataset import DeviceLoader
    from sparkmi.data.synthetic import fashion_mnist_like
    from sparkmi.models.cnn import FashionMNISTModel
    from sparkmi.ops.rng import reset_salts
    from sparkmi.optim import SGD
    from sparkmi.recipes.cnn import CNNConfig
    from sparkmi.train.trainer import Trainer
    reset_salts()
    torch.manual_seed(0)
    x, y = fashion_mnist_like(32 * 20, seed=9)
    cfg = CNNConfig(batch_size=32, lr=0.05, log_every=5, verbose=False, unroll=unroll, max_steps=steps)
    loader = DeviceLoader([x, y], 32, dev, shuffle=True, drop_last=True, seed=3, fixed=fixed)
    model = FashionMNISTModel(1, 10, 10)
    if not index:
        model.gather_in_step = lambda *a: False  # the separate gather launch (pre_step)
    tr = Trainer(model, lambda m, a, b: m.loss(a, b), lambda flat: SGD(flat, lr=cfg.lr), cfg, dev, 0, world, "t",
                 shadow=False, fused_step=lambda m, o, a, b: m.fused_sgd_step(o, a, b))
    res = tr.fit(loader, 10)
    recs = list(tr.metrics.records)
    tr.close()
    return tr.flat.master.cpu().clone(), res, recs, tr.runner


@pytest.mark.gpu
@pytest.mark.parametrize("index", [True, False])
def test_trainer_fixed_loader_multistep_graphs_bitwise(index):
    """The fixed-buffer loader's in-graph gather with 4-step graphs (and a 25-step run crossing an
    epoch boundary at 20 batches) trains bitwise the same parameters and logs the same losses as
    the per-batch gather with per-step graphs — both with the separate gather launch and with the
    fused step kernel reading the shuffled rows from the dataset itself (index mode)."""
    pa, ra, la, _ = _trainer(False, 25, 1)
    pb, rb, lb, runner = _trainer(True, 25, 4, index=index)
    assert ra["steps"] == rb["steps"] == 25
    assert (runner.pre_step is None) == index, "index mode engaged as requested"
    assert torch.equal(pa, pb)
    assert runner._multi, "the fixed loader's steps ran as multi-step graphs"
    assert [r["step"] for r in la] == [r["step"] for r in lb]
    for u, v in zip(la, lb):
        assert abs(u["loss"] - v["loss"]) <= 1e-6 * max(1.0, abs(u["loss"])), (u, v)
