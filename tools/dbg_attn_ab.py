#!/usr/bin/env python3
"""Which output differs between fp32 attention kernel variants (cross / self, modes, S): for each
toggle (row epilogue, staggered dQ + dK/dV, staggered forward) against the all-off run, print the
max |diff| per output (o, grads) — a diagnostic for tests/test_f32_gpu.py::
test_attention_f32_stagger_and_row_epilogue_bitwise."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkmi import _native  # noqa: E402
from sparkmi.ops.attention import cross_attention, self_attention  # noqa: E402

C = _native.C()
dev = "cuda"


def run(cross, mode, S):
    torch.manual_seed(13)
    B, H, hd = 2, 3, 64
    if cross:
        Sk = S + 5 if mode == "none" else S
        ins = (torch.randn(B, S, H * hd, device=dev), torch.randn(B, Sk, 128 + 2 * H * hd, device=dev))
    else:
        ins = (torch.randn(B, S, 3 * H * hd, device=dev),)
    do0 = torch.randn(B, S, H * hd, device=dev)
    xs = [t.clone().requires_grad_() for t in ins]
    o = (cross_attention(xs[0], xs[1], H, mode, kv_col=128) if cross else self_attention(xs[0], H, mode))
    o.backward(do0)
    return [o.detach()] + [t.grad.clone() for t in xs]


def setv(ae, st, fs):
    C.attn_ae(ae)
    C.attn_stagger(st)
    C.attn_fwd_stagger(fs)


for cross in (True, False):
    for mode, S in (("none", 256), ("reference", 256), ("causal", 200), ("none", 64)):
        setv(0, 0, 0)
        ref = run(cross, mode, S)
        ref2 = run(cross, mode, S)
        rep = [float((a - b).abs().max()) for a, b in zip(ref, ref2)]
        line = [f"cross={cross} {mode} S={S} repeat={rep}"]
        for name, v in (("ae", (1, 0, 0)), ("stagger", (0, 1, 0)), ("fwd8s", (0, 0, 1)), ("all", (1, 1, 1))):
            setv(*v)
            out = run(cross, mode, S)
            line.append(f"{name}=" + str([float((a - b).abs().max()) for a, b in zip(out, ref)]))
        print(" | ".join(line), flush=True)
setv(1, 1, 0)
