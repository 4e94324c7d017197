"""K-scan of the fp32 GEMM (M 8192, N 512): kernel time vs the fp32-MFMA ideal separates the
per-launch fixed cost (prologue, epilogue, launch) from the k-loop rate."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkmi.ops import gemm as G  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1000


M, N = 8192, 512
for K in [32, 128, 256, 512, 1024, 2048, 4096, 8192]:
    x, w = torch.randn(M, K, device="cuda"), torch.randn(N, K, device="cuda")
    t = timeit(lambda: G.fwd32(x, w))
    print(f"K={K:5d} {t:8.1f} us  ideal {2 * M * N * K / 157.3e6:7.1f} us", flush=True)
