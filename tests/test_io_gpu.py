"""Native input pipeline (csrc/io/pinned_ring.cpp via sparkmi.data.PinnedStreamLoader) on the GPU:
every batch equals the host rows it indexes (shuffled, several epochs, mixed dtypes) while the
consumer keeps queuing GPU work on each batch (slot / device-buffer reuse must never overwrite a
batch still in use), and the batches arrive on the compute stream without host syncs."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_pinned_ring_loader_matches_host_rows():
    from sparkmi.data.dataset import PinnedStreamLoader
    rng = np.random.default_rng(0)
    n = 1000
    imgs = rng.integers(0, 256, (n, 28, 28), dtype=np.uint8)
    feats = rng.standard_normal((n, 7)).astype(np.float32)
    labels = rng.integers(0, 10, n).astype(np.int64)
    loader = PinnedStreamLoader([imgs, feats, labels], 64, "cuda", shuffle=True, seed=5, nslots=3, threads=4)
    sums = []
    for epoch in range(3):
        order = np.random.default_rng(5 + epoch).permutation(n)
        for b, (xi, xf, y) in enumerate(loader):
            idx = order[b * 64:(b + 1) * 64]
            # heavy GPU work queued on each batch before the next one is requested
            w = torch.randn(784, 784, device="cuda")
            s = (xi.float().reshape(64, -1) @ w).sum() * 0 + xi.float().sum() + xf.sum() + y.float().sum()
            sums.append((s, float(imgs[idx].astype(np.float64).sum() + feats[idx].astype(np.float64).sum()
                                  + labels[idx].sum())))
            if b == 0:
                assert torch.equal(xi.cpu(), torch.from_numpy(imgs[idx]))
                assert torch.equal(y.cpu(), torch.from_numpy(labels[idx]))
    torch.cuda.synchronize()
    assert len(sums) == 3 * (n // 64)
    for got, want in sums:
        assert abs(float(got) - want) <= 1e-3 * abs(want) + 1e-2, (float(got), want)


def test_pinned_ring_requires_three_slots():
    from sparkmi.data.dataset import PinnedStreamLoader
    with pytest.raises(ValueError):
        PinnedStreamLoader([np.zeros((8, 2), np.float32)], 4, "cuda", nslots=2)
