"""Run one GEMM shape repeatedly (for rocprofv3 PMC collection)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparkmi.ops import gemm as G  # noqa: E402

M, N, K = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (8192, 10000, 512)))
mode = sys.argv[4] if len(sys.argv) > 4 else "fwd"
x = torch.randn(M, K, device="cuda").bfloat16()
w = torch.randn(N, K, device="cuda").bfloat16()
dy = torch.randn(M, N, device="cuda").bfloat16()
gw = torch.zeros(N, K, device="cuda")
for _ in range(20):
    if mode == "fwd":
        G.fwd(x, w)
    elif mode == "dgrad":
        G.dgrad(dy, w)
    elif mode == "blaslt":
        torch.mm(x, w.t())
    else:
        G.wgrad(dy, x, gw)
torch.cuda.synchronize()
print("done")
