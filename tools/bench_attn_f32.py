#!/usr/bin/env python3
"""fp32 attention kernels at the flagship shape (B 32, S 256, H 8, hd 64, reference mask): forward
and backward microseconds for the staged-plane kernels (default) and the per-wave split kernels
(C.attn_f32_sp(0)), plus model TFLOP/s (4 B H S^2 hd forward, 2.5x that backward).  One JSON line
per variant; ``--only sp`` runs one variant (for rocprofv3 counter passes)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkmi import _native  # noqa: E402
from sparkmi.ops.attention import self_attention  # noqa: E402


def timeit(fn, n=20, warm=3):
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
    C = _native.C()
    B, S, H, hd = 32, 256, 8, 64
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    torch.manual_seed(0)
    qkv = torch.randn(B, S, 3 * H * hd, device="cuda", requires_grad=True)
    do = torch.randn(B, S, H * hd, device="cuda")
    fl = 4.0 * B * H * S * S * hd
    for name, sp in (("staged_planes", 1), ("wave_split", 0)):
        if only and not name.startswith(only):
            continue
        C.attn_f32_sp(sp)
        fwd = timeit(lambda: self_attention(qkv.detach(), H, "reference"))

        def fb():
            o = self_attention(qkv, H, "reference")
            o.backward(do)
        tot = timeit(fb)
        bwd = tot - fwd
        print(json.dumps({"kernel": name, "fwd_us": round(fwd, 1), "bwd_us": round(bwd, 1),
                          "fwd_tf": round(fl / fwd / 1e6, 1), "bwd_tf": round(2.5 * fl / bwd / 1e6, 1)}), flush=True)
    C.attn_f32_sp(1)


if __name__ == "__main__":
    main()
