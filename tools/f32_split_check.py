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


ALGOS = (0, 6)


def group_time(C, algo, iters):
    M = 8192
    probs = [(1536, 512), (512, 512), (1024, 512), (512, 512), (512, 512), (1024, 512), (512, 1024)]
    dys = [torch.randn(M, n, device="cuda") for n, _ in probs]
    xs = [torch.randn(M, k, device="cuda") for _, k in probs]
    gws = [torch.zeros(n, k, device="cuda") for n, k in probs]
    gbs = [torch.zeros(n, device="cuda") for n, _ in probs]
    C.gemm_f32_algo(algo)

    def grp():
        C.gemm_f32_wgrad_group([d.data_ptr() for d in dys], [d.stride(0) for d in dys], [x.data_ptr() for x in xs],
                               [x.stride(0) for x in xs], [g.data_ptr() for g in gws], [b.data_ptr() for b in gbs],
                               [n for n, _ in probs], [k for _, k in probs], [M] * len(probs), _native.stream())
    t = timeit(grp, max(3, iters // 4))
    fl = sum(2 * M * n * k for n, k in probs)
    return t, fl / t / 1e6


def main(iters=20):
    C = _native.C()
    for a in ALGOS:
        t, tf = group_time(C, a, iters)
        print(f"algo{a}: wgrad group (decoder layer) {t:8.1f} us {tf:6.1f} TF/s", flush=True)
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
        for algo in ALGOS:
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
