"""Per-shape GEMM timing for the transformer's linears (M = 32*256 tokens): sparkmi MFMA kernel
vs hipBLASLt, fwd / dgrad / wgrad.  Each measurement replays a HIP graph of 20 back-to-back
launches (no host launch overhead in the number)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from sparkmi.ops import gemm as G  # noqa: E402


def gtime(fn, reps=20, iters=5):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        g.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / (iters * reps) * 1e3  # us


def main():
    M = int(os.environ.get("GEMM_M", 8192))
    shapes = [(1536, 512), (512, 512), (1024, 512), (512, 1024), (10000, 512)]
    if len(sys.argv) > 1:
        shapes = [tuple(int(v) for v in s.split("x")) for s in sys.argv[1:]]
    tot = {"smi": 0.0, "blaslt": 0.0, "best": 0.0}
    for N, K in shapes:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = torch.randn(N, K, device="cuda").bfloat16()
        dy = torch.randn(M, N, device="cuda").bfloat16()
        gw = torch.zeros(N, K, device="cuda")
        fl = 2 * M * N * K
        r = {}
        r["fwd_smi"] = gtime(lambda: G.fwd(x, w))
        r["fwd_blt"] = gtime(lambda: torch.mm(x, w.t()))
        r["dgr_smi"] = gtime(lambda: G.dgrad(dy, w))
        r["dgr_blt"] = gtime(lambda: torch.mm(dy, w))
        r["wgr_smi"] = gtime(lambda: G.wgrad(dy, x, gw))
        r["wgr_blt"] = gtime(lambda: gw.addmm_(dy.t(), x.float()) if False else torch.mm(dy.t(), x))
        line = f"N{N:6d} K{K:5d} |"
        for op in ("fwd", "dgr", "wgr"):
            a, b = r[op + "_smi"], r[op + "_blt"]
            line += f" {op} smi {a:6.1f}us {fl / a / 1e6:5.0f}TF  blt {b:6.1f}us {fl / b / 1e6:5.0f}TF |"
            tot["smi"] += a
            tot["blaslt"] += b
            tot["best"] += min(a, b)
        print(line, flush=True)
    print({k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
