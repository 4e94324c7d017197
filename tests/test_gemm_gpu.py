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


def test_wgrad_group_vs_fp32_reference():
    """Grouped no-split wgrad (csrc/kernels/gemm.hip:gemm_wgrad_group_kernel): several problems
    of different shapes in one launch — transformer shapes, ragged edges (n, k not multiples of
    128; T not a multiple of 64), strided operands, with and without the fused bias gradient —
    each accumulating onto a non-zero gradient, against fp32 torch."""
    from sparkmi import _native
    torch.manual_seed(0)
    probs = [(8192, 512, 512, True), (8192, 1536, 512, True), (8192, 512, 1024, False), (520, 200, 72, True),
             (4096, 1024, 512, True), (136, 64, 64, False)]
    As, Bs, Cs, bs, refs, brefs = [], [], [], [], [], []
    for i, (T, n, k, bias) in enumerate(probs):
        pad = 8 if i == 3 else 0  # strided rows for one problem
        a = torch.randn(T, n + pad, device=dev).bfloat16()[:, :n]
        b = torch.randn(T, k, device=dev).bfloat16()
        c = torch.randn(n, k, device=dev)
        gb = torch.randn(n, device=dev) if bias else None
        refs.append(c + a.float().t() @ b.float())
        brefs.append(gb + a.float().sum(0) if bias else None)
        As.append(a); Bs.append(b); Cs.append(c); bs.append(gb)
    _native.C().gemm_wgrad_group([a.data_ptr() for a in As], [a.stride(0) for a in As],
                                 [b.data_ptr() for b in Bs], [b.stride(0) for b in Bs], [c.data_ptr() for c in Cs],
                                 [g.data_ptr() if g is not None else 0 for g in bs], [p[1] for p in probs],
                                 [p[2] for p in probs], [p[0] for p in probs], _native.stream())
    torch.cuda.synchronize()
    for c, r, g, gr in zip(Cs, refs, bs, brefs):
        assert _rel(c, r) < 2e-5, _rel(c, r)
        if g is not None:
            assert _rel(g, gr) < 2e-5, _rel(g, gr)


def test_linear_backward_grouped_matches_per_gemm(monkeypatch):
    """A transformer backward with every wgrad queued and flushed as grouped launches gives the
    same parameter gradients as per-Linear split-K wgrads (fp32 sums in a different order)."""
    from sparkmi.models.transformer import Transformer
    from sparkmi.ops import _grad
    from sparkmi.utils.flat import FlatParams
    from sparkmi.data.synthetic import translation_pairs
    grads = []
    for group in (True, False):
        monkeypatch.setattr(_grad, "WGRAD_GROUP", group)
        torch.manual_seed(0)
        m = Transformer(d_model=256, ffn_hidden=512, num_heads=4, drop_prob=0.0, num_layers=2,
                        max_sequence_length=64, src_vocab_size=500, tgt_vocab_size=500, emb_dropout=0.0).to(dev)
        flat = FlatParams(m)
        src, tgt = translation_pairs(8, 64, 500, 500, seed=0, device=dev)
        m.training_step_loss(src, tgt).backward()
        torch.cuda.synchronize()
        assert not _grad._group_queue
        grads.append(flat.grad.clone())
    assert _rel(grads[0], grads[1]) < 1e-4, _rel(grads[0], grads[1])
