"""Split-plane fp32 GEMM (csrc/kernels/gemm_sp*.hip): operands pre-split into bf16 hi/mid/lo
planes (sparkmi/ops/planes.py).  Its error against an fp64 GEMM of the same fp32 inputs must stay
at the level of the f32-MFMA kernel (exact products, fp32 accumulation) for fwd / dgrad / wgrad
with their fused epilogues, ragged shapes, and the grouped weight-gradient launch; the planes
themselves must reconstruct their fp32 source exactly."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _err(y, ref):
    return float((y.double() - ref).norm() / ref.norm())


def _sum3(P, cols):
    return (P[0].float() + P[1].float() + P[2].float())[:, :cols]


@pytest.fixture(params=[256, 16, 128], ids=["tile256w8", "tile256m16", "tile128"])
def tile(request):
    """Every tile form of the plane GEMM (C.gemm_sp_tm: 8-wave 256 x 128, the same on the 16x16x32
    MFMA, 8-wave 128 x 128)."""
    from sparkmi import _native
    C = _native.C()
    prev = C.gemm_sp_tm(0)
    C.gemm_sp_tm(request.param)
    C.gemm_sp_wg_tm(-1)  # the grouped weight gradient follows the tile under test
    yield request.param
    C.gemm_sp_tm(prev)
    C.gemm_sp_wg_tm(-1)


@pytest.fixture
def algo():
    from sparkmi import _native
    C = _native.C()
    prev = C.gemm_f32_algo(-1)
    yield C.gemm_f32_algo
    C.gemm_f32_algo(prev)


def test_split3_exact():
    from sparkmi.ops import planes
    torch.manual_seed(0)
    for rows, cols, kpad in [(1000, 512, False), (37, 132, True), (5, 10000, True)]:
        x = torch.randn(rows, cols, device="cuda") * torch.logspace(-20, 20, cols, device="cuda")
        P = planes.split(x, kpad=kpad)
        assert P.shape[2] >= cols and (not kpad or P.shape[2] % 32 == 0)
        assert torch.equal(_sum3(P, cols), x)
        # hi is the bf16 rounding of x; the padding is zero
        assert torch.equal(P[0, :, :cols], x.to(torch.bfloat16))
        if P.shape[2] > cols:
            assert not P[:, :, cols:].any()


@pytest.mark.parametrize("M,N,K", [(1024, 512, 512), (8192, 1536, 512), (300, 264, 160), (4096, 10000, 512),
                                   (512, 1024, 1024)])
def test_sp_matches_f32_precision(algo, tile, M, N, K):
    from sparkmi.ops import gemm as G
    from sparkmi.ops import planes
    torch.manual_seed(3)
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") * 0.05
    dy = torch.randn(M, N, device="cuda")
    b = torch.randn(N, device="cuda")
    res = torch.randn(M, K, device="cuda")
    refs = {"fwd": torch.relu(x.double() @ w.double().t() + b.double()),
            "dgrad": dy.double() @ w.double() + res.double(),
            "wgrad": dy.double().t() @ x.double(), "bgrad": dy.double().sum(0)}
    assert algo(0) == 0
    gw0, gb0 = torch.zeros(N, K, device="cuda"), torch.zeros(N, device="cuda")
    out0 = {"fwd": G.fwd32(x, w, bias=b, act=1), "dgrad": G.dgrad32(dy, w, resid=res),
            "wgrad": G.wgrad32(dy, x, gw0, gb0), "bgrad": gb0}
    xp, wp = planes.split(x), planes.split(w)
    dyp = planes.split(dy, kpad=N % 32 != 0)
    y, yp = G.sp_fwd(xp, wp, M, N, K, bias=b, act=1, out_planes=True)
    dx, _ = G.sp_dgrad(dyp, wp, M, K, N, resid=res)
    gw, gb = torch.zeros(N, K, device="cuda"), torch.zeros(N, device="cuda")
    assert G.sp_wgrad(dyp, xp, gw, gb)
    torch.cuda.synchronize()
    out = {"fwd": y, "dgrad": dx, "wgrad": gw, "bgrad": gb}
    for k in refs:
        e0, e = _err(out0[k], refs[k]), _err(out[k], refs[k])
        assert e < 1e-6, (k, e, e0)
        assert e <= 1.5 * e0 + 2e-8, (k, e, e0)
    if yp is not None:  # the epilogue's planes are an exact split of its fp32 output
        assert torch.equal(_sum3(yp, N), y)


def test_sp_dgrad_dact_planes_and_dropout(tile):
    """FFN pattern: h = dropout(relu(x W1^T + b1)) with planes out; dh = (dy W2) * [h > 0] * s
    written as planes only (no fp32 copy)."""
    from sparkmi.ops import gemm as G
    from sparkmi.ops import planes
    from sparkmi.ops.rng import DropoutRNG, threshold, scale
    torch.manual_seed(1)
    M, D, F = 2048, 512, 1024
    x = torch.randn(M, D, device="cuda")
    w1 = torch.randn(F, D, device="cuda") * 0.05
    b1 = torch.randn(F, device="cuda") * 0.1
    w2 = torch.randn(D, F, device="cuda") * 0.05
    dy = torch.randn(M, D, device="cuda")
    rng = DropoutRNG(5).cuda()
    p = 0.1
    h32 = G.fwd32(x, w1, bias=b1, act=1, rng=rng, salt=7, thresh=threshold(p), dscale=scale(p))
    h, hp = G.sp_fwd(planes.split(x), planes.split(w1), M, F, D, bias=b1, act=1, rng=rng, salt=7,
                     thresh=threshold(p), dscale=scale(p), out_planes=True)
    torch.cuda.synchronize()
    # same dropout mask as the fp32 kernel, values at fp32-GEMM accuracy
    assert torch.equal(h > 0, h32 > 0) or float(((h > 0) != (h32 > 0)).float().mean()) < 1e-5
    assert torch.equal(_sum3(hp, F), h)
    ref = ((dy.double() @ w2.double()) * (h.double() > 0) * scale(p))
    dx, dhp = G.sp_dgrad(planes.split(dy), planes.split(w2), M, F, D, dact_y=h, dscale=scale(p), out_planes=True,
                         need_f32=False)
    torch.cuda.synchronize()
    assert dx is None
    assert _err(_sum3(dhp, F), ref) < 1e-6


def test_sp_wgrad_group(tile):
    from sparkmi import _native
    from sparkmi.ops import planes
    torch.manual_seed(2)
    T = 4096
    shapes = [(1536, 512), (512, 512), (1024, 512), (512, 1024), (6144, 512)]
    dys = [torch.randn(T, n, device="cuda") for n, _ in shapes]
    xs = [torch.randn(T, k, device="cuda") for _, k in shapes]
    gws = [torch.randn(n, k, device="cuda") for n, k in shapes]
    gbs = [torch.randn(n, device="cuda") for n, _ in shapes]
    refs = [(gw.double() + dy.double().t() @ x.double(), gb.double() + dy.double().sum(0))
            for gw, gb, dy, x in zip(gws, gbs, dys, xs)]
    dps = [planes.split(d) for d in dys]
    xps = [planes.split(x) for x in xs]
    _native.C().gemm_sp_wgrad_group([p.data_ptr() for p in dps], [p.stride(1) for p in dps],
                                    [p.stride(0) for p in dps], [p.data_ptr() for p in xps],
                                    [p.stride(1) for p in xps], [p.stride(0) for p in xps],
                                    [g.data_ptr() for g in gws], [g.data_ptr() for g in gbs],
                                    [n for n, _ in shapes], [k for _, k in shapes], [T] * len(shapes),
                                    _native.stream())
    torch.cuda.synchronize()
    for gw, gb, (rw, rb) in zip(gws, gbs, refs):
        assert _err(gw, rw) < 1e-6
        assert _err(gb, rb) < 1e-6
