#!/usr/bin/env python3
"""Root-cause probe for the salt-dependent one-step gradient mismatch (VERDICT r3 item 2;
tests/test_f32_gpu.py::test_transformer_f32_gradients_match_cpu_across_salts[f32mfma] fails at
salt_base 81): the L=3 concat-kv model, GPU vs CPU fp32, one step.  Reports the relative error of
decoder layer 1's FFN weights and of the gradients flowing into / out of that FFN (hooks), under
toggles: default, SMI_FFN_MASK off (fp32 hidden), grouped wgrad off, wgrad overlap off, the split
attention algorithm."""
import copy
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkmi import _native  # noqa: E402
from sparkmi.data.synthetic import translation_pairs  # noqa: E402
from sparkmi.models.transformer import Transformer  # noqa: E402
from sparkmi.ops import _grad  # noqa: E402
LIN = importlib.import_module("sparkmi.ops.linear")  # the module (sparkmi.ops.linear is also a function)
from sparkmi.utils.flat import FlatParams  # noqa: E402

C = _native.C()
dev = "cuda"
BASES = [int(b) for b in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["81"])]


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def one(base, algo, label):
    torch.manual_seed(0)
    mc = Transformer(d_model=128, ffn_hidden=256, num_heads=2, num_layers=3, max_sequence_length=32,
                     src_vocab_size=96, tgt_vocab_size=96, seed=5, dtype="fp32", salt_base=base)
    mg = copy.deepcopy(mc).to(dev)
    mc.train(); mg.train()
    FlatParams(mc)
    fg = FlatParams(mg, shadow=False)
    C.gemm_f32_algo(algo)
    src, tgt = translation_pairs(4, 32, 96, 96, seed=3)
    fg.zero_grad()
    caps = {}

    def hook(model, tag):
        ffn = model.decoder.layers[1].ffn

        def fw(mod, inp, out):
            if isinstance(out, torch.Tensor) and out.requires_grad:
                out.register_hook(lambda g, t=tag: caps.__setitem__(t + ":dy", g.detach().clone()))
            x = inp[0]
            if isinstance(x, torch.Tensor) and x.requires_grad:
                x.register_hook(lambda g, t=tag: caps.__setitem__(t + ":dx", g.detach().clone()))
        return ffn.register_forward_hook(fw)

    hc, hg = hook(mc, "c"), hook(mg, "g")
    lc = mc.training_step_loss(src, tgt)
    lg = mg.training_step_loss(src.to(dev), tgt.to(dev))
    lc.backward()
    lg.backward()
    torch.cuda.synchronize()
    hc.remove(); hg.remove()
    pc = dict(mc.named_parameters())
    pg = dict(mg.named_parameters())
    worst = max(((rel(pg[n].grad, pc[n].grad), n) for n in pc), key=lambda x: x[0])
    f = "decoder.layers.1.ffn."
    out = {"base": base, "algo": algo, "case": label, "loss_d": abs(float(lc) - float(lg)),
           "W1": rel(pg[f + "linear1.weight"].grad, pc[f + "linear1.weight"].grad),
           "b1": rel(pg[f + "linear1.bias"].grad, pc[f + "linear1.bias"].grad),
           "W2": rel(pg[f + "linear2.weight"].grad, pc[f + "linear2.weight"].grad),
           "worst": worst}
    for k in ("dy", "dx"):
        if "c:" + k in caps and "g:" + k in caps:
            out[k] = rel(caps["g:" + k], caps["c:" + k])
    print(out, flush=True)


for base in BASES:
    for algo in (0, 6):
        one(base, algo, "default")
    # toggles under the failing algorithm
    LIN._FFN_MASK = False
    one(base, 0, "ffn_mask_off")
    LIN._FFN_MASK = True
    _grad.WGRAD_GROUP = False
    one(base, 0, "wgrad_group_off")
    _grad.WGRAD_GROUP = True
    _grad.WGRAD_OVERLAP = False
    one(base, 0, "wgrad_overlap_off")
    _grad.WGRAD_OVERLAP = True
    C.attn_f32_sp(0)
    one(base, 6, "split_wave_attention")
    C.attn_f32_sp(1)
C.gemm_f32_algo(6)
