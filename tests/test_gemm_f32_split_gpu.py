"""fp32 GEMM, 3-way bf16 split algorithm (csrc/kernels/gemm_f32.hip:split3_8, SMI_F32_ALGO=6):
its error against an fp64 GEMM of the same fp32 inputs must stay at the level of the f32-MFMA
kernel (exact products, fp32 accumulation) — fwd / dgrad / wgrad, epilogues, ragged shapes."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _err(y, ref):
    return float((y.double() - ref).norm() / ref.norm())


@pytest.fixture
def algo():
    from sparkmi import _native
    C = _native.C()
    prev = C.gemm_f32_algo(-1)
    yield C.gemm_f32_algo
    C.gemm_f32_algo(prev)


@pytest.mark.parametrize("M,N,K", [(1024, 512, 512), (8192, 1536, 512), (300, 260, 132), (4096, 10000, 512)])
def test_split_matches_f32_precision(algo, M, N, K):
    from sparkmi.ops import gemm as G
    torch.manual_seed(3)
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") * 0.05
    dy = torch.randn(M, N, device="cuda")
    b = torch.randn(N, device="cuda")
    res = torch.randn(M, K, device="cuda")
    refs = {"fwd": torch.relu(x.double() @ w.double().t() + b.double()),
            "dgrad": dy.double() @ w.double() + res.double(),
            "wgrad": dy.double().t() @ x.double(), "bgrad": dy.double().sum(0)}
    errs = {}
    for a in (0, 6):
        assert algo(a) == a
        gw = torch.zeros(N, K, device="cuda")
        gb = torch.zeros(N, device="cuda")
        out = {"fwd": G.fwd32(x, w, bias=b, act=1), "dgrad": G.dgrad32(dy, w, resid=res),
               "wgrad": G.wgrad32(dy, x, gw, gb), "bgrad": gb}
        torch.cuda.synchronize()
        errs[a] = {k: _err(out[k], refs[k]) for k in refs}
    for k in refs:
        assert errs[6][k] < 1e-6, (k, errs)
        # at the f32-MFMA kernel's level (same accumulation order for the leading term)
        assert errs[6][k] <= 1.5 * errs[0][k] + 2e-8, (k, errs)
