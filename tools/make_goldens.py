#!/usr/bin/env python3
"""Generate reference-parity golden tensors from the reference's transformer.py.

Run once in the build container (the reference is mounted read-only at /root/reference and is
NOT available on the GPU box), output is checked in under tests/fixtures/ as safetensors.
The reference module is imported, never copied.  Config: d_model 128, 2 heads (head_dim 64,
the kernel's), ffn 256, 2 layers, S 16, B 3, vocab 50 -> 60; eval mode (no dropout) with the
reference's own masks (padding mask, look-ahead mask for decoder self AND cross attention).
"""
import os
import sys

import torch
from safetensors.torch import save_file

REF = os.environ.get("SPARKMI_REFERENCE", "/root/reference")
sys.path.insert(0, REF)
import transformer as ref  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures")


def main():
    torch.manual_seed(1234)
    B, S, d, H, ffn, L, Vs, Vt = 3, 16, 128, 2, 256, 2, 50, 60
    model = ref.Transformer(d, ffn, H, 0.1, L, S, Vt, list(range(Vs)), list(range(Vt)))
    model.eval()
    src = torch.randint(1, Vs, (B, S))
    tgt = torch.randint(1, Vt, (B, S))
    src[0, 10:] = 0
    tgt[1, 12:] = 0
    pad_x = (src != 0).unsqueeze(1).unsqueeze(2)
    la = (torch.tril(torch.ones(S, S)) == 0).unsqueeze(0).unsqueeze(0)
    logits = model(src, tgt, pad_x, la, la)
    lf = torch.nn.CrossEntropyLoss(ignore_index=0, reduction="none")
    loss = lf(logits.view(-1, logits.size(-1)), tgt.view(-1))
    valid = tgt.view(-1) != 0
    loss = loss[valid].sum() / valid.sum()
    loss.backward()
    tensors = {"src": src, "tgt": tgt, "logits": logits.detach(), "loss": loss.detach().reshape(1)}
    for k, v in model.state_dict().items():
        tensors["param." + k] = v.detach().clone()
    for k, p in model.named_parameters():
        tensors["grad." + k] = p.grad.detach().clone()
    # raw scaled_dot_product semantics (Q6): look-ahead mask, padding mask
    q = torch.randn(2, 4, 8, 64)
    k = torch.randn(2, 4, 8, 64)
    v = torch.randn(2, 4, 8, 64)
    la8 = (torch.tril(torch.ones(8, 8)) == 0).unsqueeze(0).unsqueeze(0)
    o_la, _ = ref.scaled_dot_product(q, k, v, la8)
    pm = torch.ones(2, 1, 1, 8, dtype=torch.bool)
    pm[0, ..., 5:] = False
    o_pm, _ = ref.scaled_dot_product(q, k, v, pm)
    tensors.update({"sdp.q": q, "sdp.k": k, "sdp.v": v, "sdp.out_lookahead": o_la, "sdp.out_padding": o_pm,
                    "pe.table": ref.PositionalEncoding(128, 16)()})
    os.makedirs(OUT, exist_ok=True)
    save_file({k: v.contiguous() for k, v in tensors.items()}, os.path.join(OUT, "transformer_ref.safetensors"))
    print("wrote", len(tensors), "tensors")


if __name__ == "__main__":
    main()
