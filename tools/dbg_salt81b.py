#!/usr/bin/env python3
"""Second root-cause probe for the salt-81 one-step mismatch (gemm_f32_algo 0 only): every fp32 /
split-plane GEMM call of the L=3 model's step is checked against an fp64 product of ITS OWN
inputs (planes reconstructed hi + mid + lo), so the first wrong kernel call is named with its
shape and epilogue flags instead of inferred from parameter gradients."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkmi import _native  # noqa: E402
from sparkmi.data.synthetic import translation_pairs  # noqa: E402
from sparkmi.models.transformer import Transformer  # noqa: E402
from sparkmi.ops import gemm as G  # noqa: E402
from sparkmi.ops import rng as _rng  # noqa: E402
from sparkmi.utils.flat import FlatParams  # noqa: E402

C = _native.C()
LOG = []


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def pl(p, rows, cols):
    return (p[0].double() + p[1].double() + p[2].double())[:rows, :cols]


def unmask(mask, M, K):
    bits = torch.stack([(mask >> e) & 1 for e in range(4)], -1).reshape(M, -1)[:, :K]
    return bits.double()


def wrap(name, fn, ref):
    def w(*a, **k):
        pre = ref(*a, **k)
        out = fn(*a, **k)
        torch.cuda.synchronize()
        got = pre(out)
        if got is not None:
            err, desc = got
            LOG.append((name, err, desc))
            flag = "  <<<<" if err > 1e-5 else ""
            print(f"{len(LOG):4d} {name:10s} rel={err:.3e} {desc}{flag}", flush=True)
        return out
    setattr(G, name, w)


def ref_dgrad32(dy, w, resid=None, dact_y=None, dscale=1.0, out=None):
    r = dy.double() @ w.double()
    if resid is not None:
        r = r + resid.double()
    if dact_y is not None:
        r = r * (dact_y.double() > 0) * dscale
    desc = f"M={dy.shape[0]} N={dy.shape[1]} K={w.shape[1]} resid={resid is not None} dact={dact_y is not None}"
    return lambda dx: (rel(dx, r), desc)


def ref_fwd32(x, w, bias=None, act=0, rng=None, salt=0, thresh=0, dscale=1.0, out=None):
    desc = f"M={x.shape[0]} N={w.shape[0]} K={x.shape[1]} act={act} drop={thresh != 0}"
    if thresh:
        return lambda y: None
    r = x.double() @ w.double().t()
    if bias is not None:
        r = r + bias.double()
    if act == 1:
        r = r.clamp_min(0)
    return lambda y: (rel(y, r), desc)


def ref_wgrad32(dy, x, gw, gb=None, splits=None):
    r = gw.double() + dy.double().t() @ x.double()
    desc = f"N={dy.shape[1]} K={x.shape[1]} M={dy.shape[0]}"
    return lambda _o: (rel(gw, r), desc)


def ref_sp_dgrad(dyp, wp, M, K, N, resid=None, dact_y=None, dscale=1.0, out_planes=False, need_f32=True, dmask=None):
    r = pl(dyp, M, N) @ pl(wp, N, K)
    if resid is not None:
        r = r + resid.double()
    if dact_y is not None:
        r = r * (dact_y.double() > 0) * dscale
    if dmask is not None:
        r = r * unmask(dmask, M, K) * dscale
    desc = f"M={M} N={N} K={K} resid={resid is not None} dact={dact_y is not None} dmask={dmask is not None} planes={out_planes} f32={need_f32}"

    def chk(o):
        if o is None:
            return 0.0, desc + " (not covered)"
        dx, dxp = o
        got = dx if dx is not None else pl(dxp, M, K)
        return rel(got, r), desc
    return chk


def ref_sp_fwd(xp, wp, M, N, K, bias=None, act=0, rng=None, salt=0, thresh=0, dscale=1.0, out_planes=False,
               lse_part=None, mask=None):
    desc = f"M={M} N={N} K={K} act={act} drop={thresh != 0} mask={mask is not None}"
    r = pl(xp, M, K) @ pl(wp, N, K).t()
    if bias is not None:
        r = r + bias.double()
    if act == 1:
        r = r.clamp_min(0)
    if thresh:
        keep = _rng.keep_mask((M, N), _rng_p(thresh), rng.current(), salt, xp.device).double()
        r = r * keep * dscale

    def chk(o):
        if o is None:
            return 0.0, desc + " (not covered)"
        y, yp = o
        got = y if y is not None else pl(yp, M, N)
        return rel(got, r), desc
    return chk


def _rng_p(thresh):
    return thresh / 2.0 ** 32


def ref_sp_wgrad(dyp, xp, gw, gb=None):
    N, K = gw.shape
    M = dyp.shape[1]
    r = gw.double() + pl(dyp, M, N).t() @ pl(xp, M, K)
    return lambda _o: (rel(gw, r), f"N={N} K={K} M={M}")


def main():
    base = int(sys.argv[1]) if len(sys.argv) > 1 else 81
    algo = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    for name, ref in (("dgrad32", ref_dgrad32), ("fwd32", ref_fwd32), ("wgrad32", ref_wgrad32),
                      ("sp_dgrad", ref_sp_dgrad), ("sp_fwd", ref_sp_fwd), ("sp_wgrad", ref_sp_wgrad)):
        wrap(name, getattr(G, name), ref)
    from sparkmi.ops import _grad
    _grad.WGRAD_GROUP = False  # standalone wgrads so each is checked
    _grad.WGRAD_OVERLAP = False
    torch.manual_seed(0)
    mc = Transformer(d_model=128, ffn_hidden=256, num_heads=2, num_layers=3, max_sequence_length=32,
                     src_vocab_size=96, tgt_vocab_size=96, seed=5, dtype="fp32", salt_base=base)
    mg = copy.deepcopy(mc).to("cuda")
    mc.train(); mg.train()
    FlatParams(mc)
    fg = FlatParams(mg, shadow=False)
    C.gemm_f32_algo(algo)
    src, tgt = translation_pairs(4, 32, 96, 96, seed=3)
    fg.zero_grad()
    lc = mc.training_step_loss(src, tgt)
    lg = mg.training_step_loss(src.cuda(), tgt.cuda())
    lc.backward()
    lg.backward()
    torch.cuda.synchronize()
    pc, pg = dict(mc.named_parameters()), dict(mg.named_parameters())
    bad = [(rel(pg[n].grad.cpu(), pc[n].grad), n) for n in pc]
    bad = sorted([b for b in bad if b[0] > 1e-4], reverse=True)
    print({"base": base, "algo": algo, "loss_d": abs(float(lc) - float(lg)), "bad_params": bad[:12]}, flush=True)
    worst = sorted(LOG, key=lambda e: -e[1])[:5]
    print("worst calls:", worst, flush=True)


if __name__ == "__main__":
    main()
