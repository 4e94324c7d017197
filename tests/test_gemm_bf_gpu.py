"""The bf16 GEMM on the 256 x 128 8-wave 16x16x32 tile (csrc/kernels/gemm_bf.hip: the split-plane
GEMM's tile with the two 32-deep k-halves of a 64-deep step as its two "planes"): exact-integer
layout checks, every epilogue against an fp32 reference and against gemm.hip's 128 x 128 kernel
(C.gemm_bf256(0)), and the grouped weight gradients (including a token count that is not a
multiple of the 64-deep k-step)."""
import pytest
import torch

from sparkmi import _native
from sparkmi.ops import gemm as G
from sparkmi.ops import rng as R

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def _both(fn):
    C = _native.C()
    prev = C.gemm_bf256(-1)
    try:
        C.gemm_bf256(1)
        new = fn()
        C.gemm_bf256(0)
        old = fn()
    finally:
        C.gemm_bf256(prev)
    return new, old


def test_bf256_layout_exact():
    """{-1, 0, 1} operands, K = 64 and 128: every sum is an integer of magnitude <= 128, exact in
    bf16; 4096 x 2048 outputs = 256 tiles of 256 x 128 (the new tile's smallest covered problem)."""
    g = torch.Generator(device=dev).manual_seed(0)
    M, N = 4096, 2048
    for K in (64, 128):
        x = torch.randint(-1, 2, (M, K), device=dev, generator=g).bfloat16()
        w = torch.randint(-1, 2, (N, K), device=dev, generator=g).bfloat16()
        y, _ = _both(lambda: G.fwd(x, w))
        assert torch.equal(y.float(), x.float() @ w.float().t())
        dy = torch.randint(-1, 2, (M, K), device=dev, generator=g).bfloat16()  # dX [M, N] from dY [M, K] W [K, N]
        wt = torch.randint(-1, 2, (K, N), device=dev, generator=g).bfloat16()
        dx, _ = _both(lambda: G.dgrad(dy, wt))
        assert torch.equal(dx.float(), dy.float() @ wt.float())


@pytest.mark.parametrize("M,N,K", [(8192, 1536, 512), (8192, 1024, 512), (8192, 10000, 512), (8192, 2048, 1024)])
@pytest.mark.parametrize("epi", ["bias", "relu", "relu_drop"])
def test_bf256_fwd_epilogues(M, N, K, epi):
    torch.manual_seed(0)
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
    b = torch.randn(N, device=dev)
    rng = R.DropoutRNG(3).to(dev)
    act = 0 if epi == "bias" else 1
    p = 0.1 if epi == "relu_drop" else 0.0
    new, old = _both(lambda: G.fwd(x, w, b, act=act, rng=rng if p else None, salt=7, thresh=R.threshold(p),
                                   dscale=R.scale(p)))
    ref = x.float() @ w.float().t() + b
    if act:
        ref = torch.relu(ref)
    if p:
        ref = ref * R.keep_mask((M, N), p, int(rng.seed.item()), 7, dev).float() * R.scale(p)
    assert _rel(new, ref) < 1e-2
    assert _rel(new, old) < 1e-2
    # identical dropout / relu zero patterns (same hash index) away from rounding-level values
    assert not ((new.float() == 0) & (ref.abs() > 1e-2)).any()
    assert not ((ref == 0) & (new.float().abs() > 1e-2)).any()


@pytest.mark.parametrize("epi", ["none", "resid", "dact", "resid_dact"])
def test_bf256_dgrad_epilogues(epi):
    torch.manual_seed(1)
    M, K, N = 8192, 2048, 512  # dX [8192, 2048]: 256 tiles
    dy = torch.randn(M, N, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
    resid = torch.randn(M, K, device=dev).bfloat16() if "resid" in epi else None
    ysave = torch.randn(M, K, device=dev).bfloat16() if "dact" in epi else None
    new, old = _both(lambda: G.dgrad(dy, w, resid=resid, dact_y=ysave, dscale=1.25))
    ref = dy.float() @ w.float()
    if resid is not None:
        ref = ref + resid.float()
    if ysave is not None:
        ref = torch.where(ysave.float() > 0, ref * 1.25, torch.zeros_like(ref))
    assert _rel(new, ref) < 1e-2
    assert _rel(new, old) < 1e-2


@pytest.mark.parametrize("T", [8192, 8200])
def test_bf256_wgrad_group(T):
    """gw_e += dY_e^T X_e and gb_e += dY_e^T 1 for a decoder layer's six weight gradients in one
    launch (> 256 tiles of 256 x 128), fp32 accumulation, tokens not a multiple of 64 included."""
    torch.manual_seed(2)
    shapes = [(1536, 512), (512, 512), (512, 512), (512, 512), (1024, 512), (512, 1024), (6144, 512)]
    dys = [torch.randn(T, n, device=dev).bfloat16() for n, _ in shapes]
    xs = [torch.randn(T, k, device=dev).bfloat16() for _, k in shapes]
    gws = [torch.randn(n, k, device=dev) for n, k in shapes]
    gbs = [torch.randn(n, device=dev) for n, _ in shapes]
    g0 = [g.clone() for g in gws]
    b0 = [b.clone() for b in gbs]

    def run():
        for g, z in zip(gws, g0):
            g.copy_(z)
        for b, z in zip(gbs, b0):
            b.copy_(z)
        _native.C().gemm_wgrad_group([d.data_ptr() for d in dys], [d.stride(0) for d in dys],
                                     [x.data_ptr() for x in xs], [x.stride(0) for x in xs],
                                     [g.data_ptr() for g in gws], [b.data_ptr() for b in gbs],
                                     [n for n, _ in shapes], [k for _, k in shapes], [T] * len(shapes),
                                     _native.stream())
        return [g.clone() for g in gws] + [b.clone() for b in gbs]

    new, old = _both(run)
    for i, (n, k) in enumerate(shapes):
        ref = dys[i].float().t() @ xs[i].float()
        assert _rel(new[i] - g0[i], ref) < 1e-4, (i, n, k)
        refb = dys[i].float().sum(0)
        assert _rel(new[len(shapes) + i] - b0[i], refb) < 1e-4, (i, "bias")
        assert _rel(new[i], old[i]) < 1e-5
