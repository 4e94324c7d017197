"""Time the fp32 GEMM (csrc/kernels/gemm_f32.hip) on the transformer's shapes: fwd / dgrad per
shape and the grouped wgrad launch of one decoder layer, reported as us and TF/s (fp32 peak
157.3 TF).  Usage: python tools/bench_gemm_f32.py [iters]"""
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


def main(iters=20):
    dev = "cuda"
    M = 8192
    rows = []
    for (N, K) in [(512, 512), (1024, 512), (1536, 512), (512, 1024), (10000, 512)]:
        x, w = torch.randn(M, K, device=dev), torch.randn(N, K, device=dev)
        t = timeit(lambda: G.fwd32(x, w), iters)
        rows.append(("fwd", M, N, K, t, 2 * M * N * K / t / 1e6))
        dy = torch.randn(M, N, device=dev)
        t = timeit(lambda: G.dgrad32(dy, w), iters)
        rows.append(("dgrad", M, K, N, t, 2 * M * N * K / t / 1e6))
    C = _native.C()
    probs = [(1536, 512), (512, 512), (1024, 512), (512, 512), (512, 512), (1024, 512), (512, 1024)]
    dys = [torch.randn(M, n, device=dev) for n, _ in probs]
    xs = [torch.randn(M, k, device=dev) for _, k in probs]
    gws = [torch.zeros(n, k, device=dev) for n, k in probs]
    gbs = [torch.zeros(n, device=dev) for n, _ in probs]

    def grp():
        C.gemm_f32_wgrad_group([d.data_ptr() for d in dys], [d.stride(0) for d in dys], [x.data_ptr() for x in xs],
                               [x.stride(0) for x in xs], [g.data_ptr() for g in gws], [b.data_ptr() for b in gbs],
                               [n for n, _ in probs], [k for _, k in probs], [M] * len(probs), _native.stream())
    t = timeit(grp, max(3, iters // 4))
    fl = sum(2 * M * n * k for n, k in probs)
    rows.append(("wgrad_group(dec layer)", M, 0, 0, t, fl / t / 1e6))
    for r in rows:
        print(f"{r[0]:24s} M={r[1]:5d} N={r[2]:5d} K={r[3]:5d}  {r[4]:9.1f} us  {r[5]:6.1f} TF/s  "
              f"{100 * r[5] / 157.3:5.1f}% of fp32 peak", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
