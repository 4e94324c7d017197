"""Time sparkmi's MFMA GEMM against hipBLASLt (torch) on the transformer's GEMM shapes."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from sparkmi.ops import gemm as G


def t(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - s) / it


def main():
    dev = "cuda"
    shapes = [(4096, 4096, 4096), (8192, 8192, 8192), (8192, 512, 512), (8192, 1536, 512), (8192, 1024, 512), (8192, 512, 1024), (8192, 10000, 512)]
    for M, N, K in shapes:
        x = torch.randn(M, K, device=dev).bfloat16()
        w = torch.randn(N, K, device=dev).bfloat16()
        dy = torch.randn(M, N, device=dev).bfloat16()
        gw = torch.zeros(N, K, device=dev)
        fl = 2 * M * N * K
        a = t(lambda: G.fwd(x, w))
        b = t(lambda: torch.mm(x, w.t()))
        c = t(lambda: G.dgrad(dy, w)) if G.supported(M, K, N, dy, w, mode=1) else float("nan")
        d = t(lambda: torch.mm(dy, w))
        e = t(lambda: G.wgrad(dy, x, gw))
        f = t(lambda: torch.mm(dy.t(), x))
        print(f"M{M} N{N} K{K}: fwd {a*1e6:7.1f}us ({fl/a/1e12:5.0f}TF) blaslt {b*1e6:7.1f}us | dgrad {c*1e6:7.1f}us "
              f"({fl/c/1e12:5.0f}TF) blaslt {d*1e6:7.1f}us | wgrad {e*1e6:7.1f}us ({fl/e/1e12:5.0f}TF) "
              f"blaslt(bf16 out) {f*1e6:7.1f}us  splits={G.wgrad_splits(N, K, M)}", flush=True)


if __name__ == "__main__":
    main()
