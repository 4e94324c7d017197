"""Run the attention forward / backward kernels of the flagship shape a few times (PMC target)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparkmi.ops.attention import self_attention  # noqa: E402

B, S, H, D = 32, 256, 8, 64
qkv = (torch.randn(B, S, 3 * H * D, device="cuda") * 0.5).bfloat16().requires_grad_()
for _ in range(5):
    out = self_attention(qkv, H, "reference", None)
    out.backward(torch.randn_like(out))
torch.cuda.synchronize()
print("ok")
