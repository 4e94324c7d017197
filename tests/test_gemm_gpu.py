"""T4: the MFMA GEMM (csrc/kernels/gemm.hip) in all three modes and every epilogue against an
fp32 torch reference, on the transformer's shapes and ragged edges."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from sparkmi.ops import gemm as G  # noqa: E402
from sparkmi.ops import rng as R  # noqa: E402

dev = "cuda"


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def test_mfma_layout_exact():
    # exact small-integer data with an asymmetric B (guide: A=I-style layout check)
    M, N, K = 128, 128, 64
    x = torch.randint(-3, 4, (M, K), device=dev).bfloat16()
    w = torch.randint(-3, 4, (N, K), device=dev).bfloat16()
    y = G.fwd(x, w)
    ref = x.float() @ w.float().t()
    assert torch.equal(y.float(), ref)
    dy = torch.randint(-3, 4, (M, N), device=dev).bfloat16()
    dx = G.dgrad(dy, w)
    assert torch.equal(dx.float(), dy.float() @ w.float())
    gw = torch.zeros(N, K, device=dev)
    G.wgrad(dy, x, gw, splits=1)
    assert torch.equal(gw, dy.float().t() @ x.float())


@pytest.mark.parametrize("M,N,K", [(8192, 512, 512), (8192, 1536, 512), (8192, 512, 1024), (8192, 1024, 512),
                                   (8192, 10000, 512), (6400, 512, 512), (200, 136, 64), (300, 200, 200),
                                   (64, 64, 4104)])
def test_fwd_shapes(M, N, K):
    torch.manual_seed(0)
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
    b = torch.randn(N, device=dev)
    y = G.fwd(x, w, b)
    ref = x.float() @ w.float().t() + b
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("M,N,K", [(8192, 512, 512), (8192, 1536, 512), (8192, 1024, 512), (6400, 512, 1024),
                                   (8192, 10000, 512), (512, 200, 72)])
def test_dgrad_wgrad(M, N, K):
    torch.manual_seed(1)
    dy = torch.randn(M, N, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
    x = torch.randn(M, K, device=dev).bfloat16()
    dx = G.dgrad(dy, w)
    assert _rel(dx, dy.float() @ w.float()) < 1e-2
    gw = torch.randn(N, K, device=dev)
    g0 = gw.clone()
    G.wgrad(dy, x, gw)
    assert _rel(gw - g0, dy.float().t() @ x.float()) < 1e-3


def test_epilogues():
    torch.manual_seed(2)
    M, N, K = 1024, 256, 128
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.1).bfloat16()
    b = torch.randn(N, device=dev)
    rng = R.DropoutRNG(9).to(dev)
    p = 0.25
    y = G.fwd(x, w, b, act=1, rng=rng, salt=5, thresh=R.threshold(p), dscale=R.scale(p))
    pre = torch.relu(x.float() @ w.float().t() + b)
    keep = R.keep_mask((M, N), p, rng.current(), 5, "cpu").to(dev)
    ref = pre * keep * R.scale(p)
    assert _rel(y, ref) < 1e-2
    # dgrad with residual and relu/dropout backward mask from y
    dy = torch.randn(M, K, device=dev).bfloat16()  # as the grad of a [M,K] output of a K->.. layer
    w2 = (torch.randn(K, N, device=dev) * 0.1).bfloat16()  # layer N -> K: weight [K, N]
    resid = torch.randn(M, N, device=dev).bfloat16()
    dh = G.dgrad(dy, w2, resid=resid, dact_y=y, dscale=R.scale(p))
    ref = (dy.float() @ w2.float() + resid.float()) * (y.float() > 0) * R.scale(p)
    assert _rel(dh, ref) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["slab", "atomic"])
@pytest.mark.parametrize("N,K,M,splits", [(512, 512, 8192, 16), (1536, 512, 2048, 3), (200, 72, 4104, 5)])
def test_wgrad_split_modes(mode, N, K, M, splits):
    torch.manual_seed(3)
    dy = torch.randn(M, N, device="cuda").bfloat16()
    x = torch.randn(M, K, device="cuda").bfloat16()
    gw = torch.randn(N, K, device="cuda")
    ref = gw + dy.float().t() @ x.float()
    old = G._WGRAD_MODE
    G._WGRAD_MODE = mode
    try:
        G.wgrad(dy, x, gw, splits=splits)
    finally:
        G._WGRAD_MODE = old
    torch.testing.assert_close(gw, ref, rtol=2e-3, atol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["slab", "atomic"])
@pytest.mark.parametrize("N,K,M,splits", [(512, 512, 8192, 16), (1536, 512, 2048, 1), (200, 72, 4104, 5)])
def test_wgrad_fused_bias_grad(mode, N, K, M, splits):
    torch.manual_seed(4)
    dy = torch.randn(M, N, device="cuda").bfloat16()
    x = torch.randn(M, K, device="cuda").bfloat16()
    gw = torch.zeros(N, K, device="cuda")
    gb = torch.randn(N, device="cuda")
    ref_b = gb + dy.float().sum(0)
    old = G._WGRAD_MODE
    G._WGRAD_MODE = mode
    try:
        G.wgrad(dy, x, gw, splits=splits, gb=gb)
    finally:
        G._WGRAD_MODE = old
    torch.testing.assert_close(gw, dy.float().t() @ x.float(), rtol=2e-3, atol=2e-2)
    torch.testing.assert_close(gb, ref_b, rtol=1e-3, atol=2e-2)
