"""Time one LSTM training step (reference config: V~95k, H=32, L=2, B=32, T=129) on the fused kernels."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparkmi.models.lstm import LSTM  # noqa: E402
from sparkmi.optim import Adam  # noqa: E402
from sparkmi.utils.flat import FlatParams  # noqa: E402

V, B, T = 95812, 32, 129
m = LSTM(V, 32, 32, 4, num_layers=2, padding_idx=7).cuda().train()
flat = FlatParams(m, shadow=False)
opt = Adam(flat, lr=1e-3)
ids = torch.randint(0, V, (B, T), device="cuda")
y = torch.randint(0, 4, (B,), device="cuda")


def step():
    loss, _ = m.loss(ids, y)
    loss.backward()
    opt.step()
    m.rng.advance()


for _ in range(5):
    step()
torch.cuda.synchronize()
n = 50
t = time.perf_counter()
for _ in range(n):
    step()
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / n
print(f"lstm step {dt*1e3:.3f} ms  -> {B/dt:.0f} samples/s")
