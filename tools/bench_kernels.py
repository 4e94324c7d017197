"""Microbenchmarks of sparkmi's non-GEMM HIP kernels at the flagship transformer shapes
(M = 32*256 tokens, d = 512, H = 8, S = 256): HIP-event timing, achieved bandwidth/FLOPs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparkmi import _native  # noqa: E402
from sparkmi.ops import rng as R  # noqa: E402


def timeit(fn, reps=20, it=5):
    """Replay a HIP graph of `reps` back-to-back launches: device time per launch, no host overhead."""
    fn()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        g.replay()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / (reps * it) * 1000  # us


def main():
    C = _native.C()
    st = lambda: _native.stream()  # noqa: E731
    dev = "cuda"
    M, D = 8192, 512
    h = torch.randn(M, D, device=dev).bfloat16()
    r = torch.randn(M, D, device=dev).bfloat16()
    g = torch.ones(D, device=dev)
    b = torch.zeros(D, device=dev)
    y, xs = torch.empty_like(h), torch.empty_like(h)
    mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
    seed = torch.zeros(1, dtype=torch.int32, device=dev)
    thr = R.threshold(0.1)
    t = timeit(lambda: C.ln_fwd(h.data_ptr(), r.data_ptr(), g.data_ptr(), b.data_ptr(), y.data_ptr(), xs.data_ptr(),
                                mean.data_ptr(), rstd.data_ptr(), M, D, 1e-5, seed.data_ptr(), 7, thr, 1.1, st()))
    print(f"ln_fwd      {t:8.1f} us  {4 * M * D * 2 / t / 1e3:7.0f} GB/s")
    part = torch.empty(2, 2048, D, device=dev)
    dres, dh = torch.empty_like(h), torch.empty_like(h)
    t = timeit(lambda: C.ln_bwd(h.data_ptr(), xs.data_ptr(), mean.data_ptr(), rstd.data_ptr(), g.data_ptr(),
                                dres.data_ptr(), dh.data_ptr(), 0, part[0].data_ptr(), part[1].data_ptr(), 2048,
                                g.data_ptr(), b.data_ptr(), 1, M, D, seed.data_ptr(), 7, thr, 1.1, st()))
    print(f"ln_bwd      {t:8.1f} us  {4 * M * D * 2 / t / 1e3:7.0f} GB/s")
    out = torch.zeros(D, device=dev)
    for rpb in (32, 64, 256):
        t = timeit(lambda: C.colsum_bf16(h.data_ptr(), M, D, 0, rpb, out.data_ptr(), 1, st()))
        print(f"colsum rpb{rpb:4d} {t:8.1f} us  {M * D * 2 / t / 1e3:7.0f} GB/s")
    from sparkmi.ops.attention import _AttnCore  # noqa: F401
    import math
    B, S, H = 32, 256, 8
    qkv = torch.randn(B, S, 3 * H * 64, device=dev).bfloat16()
    o = torch.empty(B, S, H * 64, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, S, device=dev)
    qs = (S * 3 * H * 64, 3 * H * 64, 3 * 64)
    os_ = (S * H * 64, H * 64, 64)
    base = qkv.data_ptr()
    for mode in (0, 1, 2):
        t = timeit(lambda: C.attn_fwd(base, base + 128, base + 256, qs, qs, qs, o.data_ptr(), os_, lse.data_ptr(), 0,
                                      B, H, S, S, mode, 1.4426950408889634 / 8, st()))
        fl = 4 * B * H * S * S * 64 * (0.5 if mode == 2 else 1)
        print(f"attn_fwd m{mode} {t:8.1f} us  {fl / t / 1e6:7.0f} TF")
    do = torch.randn_like(o)
    dqkv = torch.empty_like(qkv)
    delta = torch.empty(B, H, S, device=dev)
    for mode in (0, 1):
        t = timeit(lambda: C.attn_bwd(base, base + 128, base + 256, qs, qs, qs, o.data_ptr(), do.data_ptr(), os_,
                                      lse.data_ptr(), delta.data_ptr(), dqkv.data_ptr(), dqkv.data_ptr() + 128,
                                      dqkv.data_ptr() + 256, 0, B, H, S, S, mode, 1.4426950408889634 / 8, 0.125, st()))
        print(f"attn_bwd m{mode} {t:8.1f} us  {10 * B * H * S * S * 64 / t / 1e6:7.0f} TF (5-GEMM count)")
    V = 10000
    logits = torch.randn(M, V, device=dev).bfloat16()
    lab = torch.randint(0, V, (M,), device=dev)
    lse2 = torch.empty(M, device=dev)
    stats = torch.empty(2, device=dev)
    rl = torch.empty(M, device=dev)
    t = timeit(lambda: C.ce_fwd(logits.data_ptr(), 1, lab.data_ptr(), M, V, 0, lse2.data_ptr(), stats.data_ptr(),
                                stats.data_ptr() + 4, rl.data_ptr(), st()))
    print(f"ce_fwd      {t:8.1f} us  {M * V * 2 / t / 1e3:7.0f} GB/s")
    grad = torch.empty_like(logits)
    dl = torch.ones(1, device=dev)
    t = timeit(lambda: C.ce_bwd(logits.data_ptr(), 1, lab.data_ptr(), M, V, 0, lse2.data_ptr(), stats.data_ptr(),
                                dl.data_ptr(), grad.data_ptr(), 0, 0, 0, st()))
    print(f"ce_bwd      {t:8.1f} us  {2 * M * V * 2 / t / 1e3:7.0f} GB/s")
    n = 47_000_000
    p_, g_, m_, v_ = (torch.randn(n, device=dev) for _ in range(4))
    pb = torch.empty(n, device=dev, dtype=torch.bfloat16)
    lr, stp = torch.full((1,), 1e-3, device=dev), torch.ones(1, device=dev)
    done = torch.zeros(1, device=dev, dtype=torch.int32)
    t = timeit(lambda: C.adam(p_.data_ptr(), g_.data_ptr(), m_.data_ptr(), v_.data_ptr(), pb.data_ptr(), n,
                              lr.data_ptr(), stp.data_ptr(), done.data_ptr(), 0.9, 0.999, 1e-8, 0.0, 1.0, 0, 1, 0, 0, 0, st()))
    print(f"adam 47M    {t:8.1f} us  {n * (4 * 4 + 4 * 4 + 2) / t / 1e3:7.0f} GB/s")
    ids = torch.randint(0, V, (M,), device=dev)
    table = torch.randn(V, D, device=dev).bfloat16()
    pe = torch.randn(S, D, device=dev)
    eo = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: C.emb_fwd(ids.data_ptr(), table.data_ptr(), pe.data_ptr(), eo.data_ptr(), M, D, S,
                                 seed.data_ptr(), 3, thr, 1.1, st()))
    print(f"emb_fwd     {t:8.1f} us")
    dt = torch.zeros(V, D, device=dev)
    ews = torch.empty(C.emb_det_ws_bytes(M, V, D), device=dev, dtype=torch.uint8)
    for det in (0, 1):
        t = timeit(lambda: C.emb_bwd(ids.data_ptr(), eo.data_ptr(), dt.data_ptr(), M, D, -1, seed.data_ptr(), 3, thr,
                                     1.1, V, ews.data_ptr() if det else 0, st()))
        print(f"emb_bwd {'bucketed' if det else 'atomic'} {t:8.1f} us")


if __name__ == "__main__":
    main()
