"""Deferred backward work (sparkmi/ops/_grad.py) with a module REUSED within one forward: a
Linear whose weight is queued twice for the grouped wgrad launch and a LayerNormalization whose
dgamma/dbeta folds are queued twice must give the same gradients as the immediate (non-deferred)
paths — the batch split on a repeated output pointer is what prevents the lost-update race —
and so must the in-op early flush once the queued-bytes cap is exceeded.  fp32 and bf16."""
import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu
dev = "cuda"


class Reuse(nn.Module):
    def __init__(self, d, dtype):
        super().__init__()
        from sparkmi.models.transformer import LayerNormalization
        self.lin = nn.Linear(d, d)
        self.ln = LayerNormalization([d])
        self.head = nn.Linear(d, d)
        self.dtype = dtype

    def forward(self, x):
        from sparkmi.ops.linear import linear
        h = linear(x, self.lin.weight, self.lin.bias)
        h = self.ln(h, x)
        h2 = linear(h, self.lin.weight, self.lin.bias)  # same Linear again
        h2 = self.ln(h2, h)                             # same LayerNorm again
        return linear(h2, self.head.weight, self.head.bias)


def _grads(dtype, group, ln_defer, fold_defer, cap, monkeypatch):
    from sparkmi.ops import _grad
    from sparkmi.utils.flat import FlatParams
    monkeypatch.setattr(_grad, "WGRAD_GROUP", group)
    monkeypatch.setattr(_grad, "LN_DEFER", ln_defer)
    monkeypatch.setattr(_grad, "FOLD_DEFER", fold_defer)
    monkeypatch.setattr(_grad, "GROUP_CAP_BYTES", cap)
    torch.manual_seed(0)
    m = Reuse(256, dtype).to(dev)
    flat = FlatParams(m, shadow=(dtype == "bf16"))
    x = torch.randn(1024, 256, device=dev)
    if dtype == "bf16":
        x = x.bfloat16()
    y = m(x)
    (y.float() ** 2).mean().backward()
    torch.cuda.synchronize()
    assert not _grad.pending()
    return flat.grad.clone()


@pytest.mark.parametrize("dtype", ["fp32"])
def test_reused_modules_deferred_equal_immediate(dtype, monkeypatch):
    ref = _grads(dtype, False, False, False, 1 << 40, monkeypatch)
    deferred = _grads(dtype, True, True, True, 1 << 40, monkeypatch)
    capped = _grads(dtype, True, True, True, 1, monkeypatch)  # flush from inside every queued op
    scale = ref.abs().max()
    assert float((deferred - ref).abs().max() / scale) < 1e-5
    assert float((capped - ref).abs().max() / scale) < 1e-5
