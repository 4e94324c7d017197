#!/usr/bin/env python3
"""The fp32 LayerNorm forward at the transformer's shape (8192 x 512, residual, dropout 0.1, split
planes out: 88 MB) against a plain torch copy of the same byte count, interleaved rounds — is the
kernel at HBM speed?  (Round 5: 16.4 us vs 16.2 us for the copy, profiles/r5_ab_ln_rows.txt.)  Also
times the backward (fp32: dres + dh planes, bf16: dres + dh).
Usage (GPU box): python tools/ab_ln.py"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    import torch
    from sparkmi import _native
    from sparkmi.ops import rng as R
    C = _native.C()
    M, D = 8192, 512
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    h = torch.randn(M, D, generator=g).to(dev)
    r = torch.randn(M, D, generator=g).to(dev)
    gam = (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
    bet = (0.1 * torch.randn(D, generator=g)).to(dev)
    seed = torch.tensor([1234], dtype=torch.int32, device=dev)
    y, xs = torch.empty_like(h), torch.empty_like(h)
    mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
    planes = torch.empty(3, M, D, device=dev, dtype=torch.bfloat16)
    st = _native.stream()

    def fwd():
        C.ln_fwd_f32(h.data_ptr(), r.data_ptr(), gam.data_ptr(), bet.data_ptr(), y.data_ptr(), xs.data_ptr(),
                     mean.data_ptr(), rstd.data_ptr(), M, D, 1e-5, seed.data_ptr(), 7, R.threshold(0.1), R.scale(0.1),
                     planes.data_ptr(), planes.stride(0), st)

    def timeit(fn):
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.iters

    # backward, fp32 (planes-only dh) and bf16
    dy = torch.randn(M, D, generator=g).to(dev)
    dres = torch.empty_like(dy)
    part = torch.empty(2, M // 4, D, device=dev)
    dhp = torch.empty(3, M, D, device=dev, dtype=torch.bfloat16)
    dyb, xsb = dy.bfloat16(), xs.bfloat16()
    dresb, dhb = torch.empty_like(dyb), torch.empty_like(dyb)

    def bwd32():
        C.ln_bwd_f32(dy.data_ptr(), xs.data_ptr(), mean.data_ptr(), rstd.data_ptr(), gam.data_ptr(), dres.data_ptr(),
                     0, 0, part[0].data_ptr(), part[1].data_ptr(), M // 4, 0, 0, 1, M, D, seed.data_ptr(), 7,
                     R.threshold(0.1), R.scale(0.1), dhp.data_ptr(), dhp.stride(0), st)

    def bwd16():
        C.ln_bwd(dyb.data_ptr(), xsb.data_ptr(), mean.data_ptr(), rstd.data_ptr(), gam.data_ptr(), dresb.data_ptr(),
                 dhb.data_ptr(), 0, part[0].data_ptr(), part[1].data_ptr(), M // 4, 0, 0, 1, M, D, seed.data_ptr(), 7,
                 R.threshold(0.1), R.scale(0.1), st)

    for rd in range(a.rounds):
        print(f"round {rd}: ln_bwd fp32 (dres + dh planes) {timeit(bwd32):6.2f} us | bf16 {timeit(bwd16):6.2f} us",
              flush=True)
    src = torch.empty(32 * (1 << 20) // 4, device=dev)
    dst = torch.empty(56 * (1 << 20) // 4, device=dev)
    nbytes = M * D * 4 * 2 + M * D * 4 * 2 + M * D * 2 * 3
    for rd in range(a.rounds):
        t = timeit(fwd)
        line = [f"ln_fwd {t:6.2f} us ({nbytes / t / 1e3:5.0f} GB/s)"]
        tc = timeit(lambda: (dst[: src.numel()].copy_(src), dst[src.numel():].copy_(src[: dst.numel() - src.numel()])))
        line.append(f"torch copy 88 MB {tc:6.2f} us")
        print(f"round {rd}: " + " | ".join(line), flush=True)


if __name__ == "__main__":
    main()
