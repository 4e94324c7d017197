"""Peak HBM of one flagship training step (transformer L6 d512 S256 batch 32) with the grouped
weight-gradient queue on and off (sparkmi/ops/_grad.py WGRAD_GROUP, and with a small queue cap),
fp32 and bf16: torch.cuda.max_memory_allocated around forward + backward + optimizer."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkmi.data.synthetic import translation_pairs  # noqa: E402
from sparkmi.models.transformer import Transformer  # noqa: E402
from sparkmi.ops import _grad  # noqa: E402
from sparkmi.optim import Adam  # noqa: E402
from sparkmi.utils.flat import FlatParams  # noqa: E402


def peak(dtype, group, cap_mb):
    _grad.WGRAD_GROUP = group
    _grad.GROUP_CAP_BYTES = int(cap_mb * (1 << 20))
    torch.manual_seed(0)
    m = Transformer(d_model=512, ffn_hidden=1024, num_heads=8, drop_prob=0.1, num_layers=6, max_sequence_length=256,
                    src_vocab_size=10000, tgt_vocab_size=10000, dtype=dtype).cuda().train()
    flat = FlatParams(m, shadow=dtype == "bf16")
    opt = Adam(flat, lr=1e-3)
    src, tgt = translation_pairs(32, 256, 10000, 10000, seed=0, device="cuda")
    for _ in range(2):
        m.rng.advance()
        loss = m.training_step_loss(src, tgt)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    m.rng.advance()
    loss = m.training_step_loss(src, tgt)
    loss.backward()
    opt.step()
    torch.cuda.synchronize()
    pk = torch.cuda.max_memory_allocated()
    del m, flat, opt, loss
    torch.cuda.empty_cache()
    return round((pk - base) / 2**20, 1), round(pk / 2**20, 1)


def main():
    rows = []
    for dtype in ("fp32", "bf16"):
        for group, cap in ((False, 8192), (True, 8192), (True, 256)):
            step_mb, total_mb = peak(dtype, group, cap)
            rows.append({"dtype": dtype, "wgrad_group": group, "cap_mb": cap, "step_peak_over_resident_mb": step_mb,
                         "peak_allocated_mb": total_mb})
            print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
