#!/usr/bin/env python3
"""Timing / A/B of the attention kernels at the flagship shape (B 32, S 256, H 8, hd 64,
reference mask, planes out as in the model): single-pass backward vs the dQ + dK/dV pair
(C.attn_bwd1) and, in fp32, the whole-row LDS epilogue on/off (C.attn_ae).  Each variant is timed
in interleaved rounds (forward alone, then forward + backward) so clock drift hits every variant
alike; one JSON line per variant with the median over rounds.  --dtype bf16 times the bf16 kernels."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkmi import _native  # noqa: E402
from sparkmi.ops import planes as PL  # noqa: E402
from sparkmi.ops.attention import self_attention  # noqa: E402


def timeit(fn, n=30):
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
    torch.manual_seed(0)
    bf16 = "--dtype" in sys.argv and sys.argv[sys.argv.index("--dtype") + 1] == "bf16"
    dt = torch.bfloat16 if bf16 else torch.float32
    qkv = torch.randn(B, S, 3 * H * hd, device="cuda", dtype=dt, requires_grad=True)
    do = torch.randn(B, S, H * hd, device="cuda", dtype=dt)
    if not bf16:
        PL.attach(do, PL.split(do.reshape(-1, H * hd)))
    variants = [("single_pass", 1, 1), ("pair", 1, 0)] + ([] if bf16 else [("single_pass_per_lane", 0, 1)])
    if "--only" in sys.argv:
        only = sys.argv[sys.argv.index("--only") + 1]
        variants = [v for v in variants if v[0] == only]
    res = {v[0]: ([], []) for v in variants}
    for _ in range(5):
        for name, ae, b1 in variants:
            C.attn_ae(ae)
            C.attn_bwd1(b1)
            f = timeit(lambda: self_attention(qkv.detach(), H, "reference"))

            def fb():
                o = self_attention(qkv, H, "reference")
                o.backward(do)
            t = timeit(fb)
            res[name][0].append(f)
            res[name][1].append(t - f)
    fl = 4.0 * B * H * S * S * hd
    for name, (fs, bs) in res.items():
        f, b = statistics.median(fs), statistics.median(bs)
        print(json.dumps({"variant": name, "dtype": "bf16" if bf16 else "fp32", "fwd_us": round(f, 1), "bwd_us": round(b, 1),
                          "fwd_tf": round(fl / f / 1e6, 1), "bwd_tf": round(2.5 * fl / b / 1e6, 1)}), flush=True)
    C.attn_ae(1)
    C.attn_bwd1(1)


if __name__ == "__main__":
    main()
