#!/usr/bin/env python3
"""sparkmi's bf16 GEMM (csrc/kernels/gemm.hip) vs hipBLASLt (torch.matmul) on the transformer's
shapes (M = 8192 tokens): forward, dgrad, and the weight gradient (fp32 accumulate; hipBLASLt
writes a bf16/fp32 product without the accumulate, an upper bound).  One JSON line per shape:
microseconds and TFLOP/s (2 M N K / t)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkmi.ops import gemm as G  # noqa: E402


def timeit(fn, n=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / n


def main():
    M = 8192
    bf = torch.bfloat16
    for N, K in [(512, 512), (1536, 512), (1024, 512), (512, 1024), (6144, 512), (10000, 512)]:
        x = torch.randn(M, K, device="cuda", dtype=bf)
        w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
        b = torch.randn(N, device="cuda")
        dy = torch.randn(M, N, device="cuda", dtype=bf)
        gw = torch.zeros(N, K, device="cuda")
        fl = 2.0 * M * N * K
        r = {"N": N, "K": K}
        r["fwd_us"] = timeit(lambda: G.fwd(x, w, bias=b))
        r["dgrad_us"] = timeit(lambda: G.dgrad(dy, w))
        r["wgrad_us"] = timeit(lambda: G.wgrad(dy, x, gw))
        r["blas_fwd_us"] = timeit(lambda: torch.matmul(x, w.t()))
        r["blas_dgrad_us"] = timeit(lambda: torch.matmul(dy, w))
        r["blas_wgrad_us"] = timeit(lambda: torch.matmul(dy.t(), x))
        for k in list(r):
            if k.endswith("_us"):
                r[k.replace("_us", "_tf")] = round(fl / (r[k] * 1e-6) / 1e12, 1)
                r[k] = round(r[k], 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
