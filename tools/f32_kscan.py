import sys, torch
sys.path.insert(0, "/root/repo")
from sparkmi.ops import gemm as G
def timeit(fn, iters=20):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters): fn()
    e.record(); e.synchronize()
    return s.elapsed_time(e) / iters * 1000
M, N = 8192, 512
for K in [128, 256, 512, 1024, 2048, 4096, 8192]:
    x, w = torch.randn(M, K, device="cuda"), torch.randn(N, K, device="cuda")
    t = timeit(lambda: G.fwd32(x, w))
    print(f"K={K:5d} {t:8.1f} us  ideal {2*M*N*K/157.3e6:7.1f} us", flush=True)
# zero data (clock check)
K=4096
x, w = torch.zeros(M, K, device="cuda"), torch.zeros(N, K, device="cuda")
print("zeros K=4096", timeit(lambda: G.fwd32(x, w)))
