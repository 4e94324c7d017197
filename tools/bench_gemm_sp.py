#!/usr/bin/env python3
"""Split-plane fp32 GEMM vs the split-inside-the-GEMM fp32 kernel (algo 6) and f32 MFMA (algo 0)
on the transformer's shapes (M = 8192 tokens): fwd, dgrad, and one decoder layer's grouped
wgrad.  Prints microseconds per launch and the model TFLOP/s (2 M N K / t)."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from sparkmi import _native  # noqa: E402
from sparkmi.ops import gemm as G  # noqa: E402
from sparkmi.ops import planes  # noqa: E402


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
    M = 8192
    rows = []
    shapes = [(512, 512), (1536, 512), (1024, 512), (512, 1024), (6144, 512), (10000, 512)]
    for N, K in shapes:
        x = torch.randn(M, K, device="cuda")
        w = torch.randn(N, K, device="cuda") * 0.05
        b = torch.randn(N, device="cuda")
        dy = torch.randn(M, N, device="cuda")
        xp, wp = planes.split(x), planes.split(w)
        dyp = planes.split(dy, kpad=N % 32 != 0)
        fl = 2.0 * M * N * K
        r = {"N": N, "K": K}
        gw = torch.zeros(N, K, device="cuda")
        for tm in (16, 256, 128):
            C.gemm_sp_tm(tm)
            r[f"sp{tm}_fwd_us"] = timeit(lambda: G.sp_fwd(xp, wp, M, N, K, bias=b))
            r[f"sp{tm}_dgrad_us"] = timeit(lambda: G.sp_dgrad(dyp, wp, M, K, N))
            r[f"sp{tm}_wgrad_us"] = timeit(lambda: G.sp_wgrad(dyp, xp, gw))
        C.gemm_sp_tm(16)
        r["split_x_us"] = timeit(lambda: planes.split(x))
        r["split_dy_us"] = timeit(lambda: planes.split(dy, kpad=N % 32 != 0))
        for a in ((6, 0) if "--f32" in sys.argv else ()):
            C.gemm_f32_algo(a)
            r[f"a{a}_fwd_us"] = timeit(lambda: G.fwd32(x, w, bias=b))
            r[f"a{a}_dgrad_us"] = timeit(lambda: G.dgrad32(dy, w))
        C.gemm_f32_algo(6)
        for k in list(r):
            if k.endswith("_us") and not k.startswith("split"):
                r[k.replace("_us", "_tf")] = round(fl / (r[k] * 1e-6) / 1e12, 1)
        r = {k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}
        rows.append(r)
        print(json.dumps(r), flush=True)
    # one decoder layer's weight gradients as one grouped launch
    T = M
    shp = [(1536, 512), (512, 512), (512, 512), (512, 512), (1024, 512), (512, 1024)]
    dys = [planes.split(torch.randn(T, n, device="cuda")) for n, _ in shp]
    xs = [planes.split(torch.randn(T, k, device="cuda")) for _, k in shp]
    gws = [torch.zeros(n, k, device="cuda") for n, k in shp]
    gbs = [torch.zeros(n, device="cuda") for n, _ in shp]

    def grp():
        C.gemm_sp_wgrad_group([p.data_ptr() for p in dys], [p.stride(1) for p in dys], [p.stride(0) for p in dys],
                              [p.data_ptr() for p in xs], [p.stride(1) for p in xs], [p.stride(0) for p in xs],
                              [g.data_ptr() for g in gws], [g.data_ptr() for g in gbs], [n for n, _ in shp],
                              [k for _, k in shp], [T] * len(shp), _native.stream())
    fl = sum(2.0 * T * n * k for n, k in shp)
    for tm in (16, 256, 128):
        C.gemm_sp_tm(tm)
        t = timeit(grp)
        print(json.dumps({f"sp{tm}_wgrad_group_dec_layer_us": round(t, 1), "tf": round(fl / (t * 1e-6) / 1e12, 1)}),
              flush=True)
    C.gemm_sp_tm(16)


if __name__ == "__main__":
    main()
