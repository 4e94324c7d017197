#!/usr/bin/env python3
"""The bf16 matrix-core rate this MI355X sustains on RANDOM data — the practical ceiling of any
GEMM built from v_mfma_f32_32x32x16_bf16, including the fp32 split-plane GEMM (6 bf16 products per
fp32 product, so its ceiling is this rate / 6).  Under load the chip lowers its clock on random
operands (docs: MI355X_MICROARCH "DVFS give-back"), so the 2.5 PF spec is not reachable; this
measures hipBLASLt (torch.matmul) and sparkmi's own bf16 GEMM on large square shapes, random and
all-zero inputs (the zero run shows the clock headroom).  Prints one JSON line per case."""
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
    return e0.elapsed_time(e1) / 1e3 / n


def main():
    for n in (8192, 16384):
        fl = 2.0 * n ** 3
        for kind in ("random", "zeros"):
            mk = torch.randn if kind == "random" else torch.zeros
            a = mk(n, n, device="cuda", dtype=torch.bfloat16)
            b = mk(n, n, device="cuda", dtype=torch.bfloat16)
            t = timeit(lambda: torch.matmul(a, b))
            row = {"shape": n, "data": kind, "hipblaslt_tf": round(fl / t / 1e12, 1)}
            if G.supported(n, n, n, a, b, mode=0):
                t2 = timeit(lambda: G.fwd(a, b))  # y = a @ b^T on sparkmi's bf16 kernel
                row["sparkmi_bf16_tf"] = round(fl / t2 / 1e12, 1)
            row["fp32_split_ceiling_tf"] = round(max(v for k, v in row.items() if k.endswith("_tf")) / 6, 1)
            print(json.dumps(row), flush=True)
            del a, b
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
