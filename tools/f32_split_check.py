"""fp32 GEMM product algorithms side by side: f32 MFMA (algo 0) vs the 3-way bf16 split with 6
product terms (algo 6, csrc/kernels/gemm_f32.hip:split3_8).  For each transformer shape: error
against an fp64 GEMM of the same fp32 inputs (max |err| / max |ref| and RMS relative error) and
time / TF/s of both.  Usage: python tools/f32_split_check.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkmi import _native  # noqa: E402
from sparkmi.ops import gemm as G  # noqa: E402


def timeit(fn, iters):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def err(y, ref):
    d = (y.double() - ref)
    return float(d.abs().max() / ref.abs().max()), float(d.norm() / ref.norm())


def main(iters=20):
    C = _native.C()
    dev = "cuda"
    M = 8192
    torch.manual_seed(0)
    for (N, K) in [(512, 512), (1024, 512), (1536, 512), (512, 1024), (10000, 512)]:
        x, w = torch.randn(M, K, device=dev), torch.randn(N, K, device=dev) * 0.05
        dy = torch.randn(M, N, device=dev)
        ref_f = x.double() @ w.double().t()
        ref_d = dy.double() @ w.double()
        ref_w = dy.double().t() @ x.double()
        line = []
        for algo in (0, 6):
            C.gemm_f32_algo(algo)
            yf = G.fwd32(x, w)
            yd = G.dgrad32(dy, w)
            gw = torch.zeros(N, K, device=dev)
            G.wgrad32(dy, x, gw)
            torch.cuda.synchronize()
            tf = timeit(lambda: G.fwd32(x, w), iters)
            td = timeit(lambda: G.dgrad32(dy, w), iters)
            fl = 2 * M * N * K
            line.append(f"algo{algo}: fwd {tf:7.1f}us {fl / tf / 1e6:6.1f}TF err {err(yf, ref_f)[0]:.2e}/{err(yf, ref_f)[1]:.2e}"
                        f" | dgrad {td:7.1f}us {fl / td / 1e6:6.1f}TF err {err(yd, ref_d)[0]:.2e}/{err(yd, ref_d)[1]:.2e}"
                        f" | wgrad err {err(gw, ref_w)[0]:.2e}/{err(gw, ref_w)[1]:.2e}")
        print(f"M={M} N={N} K={K}", flush=True)
        for ln in line:
            print("   " + ln, flush=True)
    C.gemm_f32_algo(0)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
