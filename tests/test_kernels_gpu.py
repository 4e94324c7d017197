"""T4: every HIP kernel against the fp32 torch reference path of the same op (same dropout
mask via the shared counter-based hash).  Runs on an MI355X only."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from sparkmi import _native  # noqa: E402
from sparkmi.ops import rng as R  # noqa: E402
from sparkmi.ops.attention import cross_attention, self_attention  # noqa: E402
from sparkmi.ops.embedding import embedding, sinusoid_table  # noqa: E402
from sparkmi.ops.layernorm import add_dropout_layernorm  # noqa: E402
from sparkmi.ops.linear import linear  # noqa: E402
from sparkmi.ops.loss import cross_entropy  # noqa: E402

dev = "cuda"


def _close(a, b, atol, rtol, msg=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol)
    assert not bad.any(), f"{msg}: {bad.sum().item()} / {bad.numel()} mismatches, max err {err.max().item():.4g}"


def test_native_loaded():
    C = _native.C()
    assert C.ARCH == "gfx950"
    assert "_C" in C.__file__


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_layernorm(p):
    torch.manual_seed(0)
    M, D = 1000, 512
    rng_g, rng_c = R.DropoutRNG(7).to(dev), R.DropoutRNG(7)
    h = torch.randn(M, D)
    r = torch.randn(M, D)
    gamma = torch.nn.Parameter(torch.randn(D) * 0.5 + 1)
    beta = torch.nn.Parameter(torch.randn(D) * 0.1)
    gamma_g = torch.nn.Parameter(gamma.detach().to(dev))
    beta_g = torch.nn.Parameter(beta.detach().to(dev))
    hb, rb = h.bfloat16(), r.bfloat16()
    hg = hb.to(dev).requires_grad_()
    rg = rb.to(dev).requires_grad_()
    hc = hb.float().requires_grad_()
    rc = rb.float().requires_grad_()
    yg = add_dropout_layernorm(hg, rg, gamma_g, beta_g, p, rng_g, 1234)
    yc = add_dropout_layernorm(hc, rc, gamma, beta, p, rng_c, 1234)
    _close(yg, yc, 3e-2, 2e-2, "ln fwd")
    dy = torch.randn(M, D).bfloat16()
    yg.backward(dy.to(dev))
    yc.backward(dy.float())
    _close(hg.grad, hc.grad, 3e-2, 3e-2, "dh")
    _close(rg.grad, rc.grad, 3e-2, 3e-2, "dres")
    _close(gamma_g.grad, gamma.grad, 0.5, 2e-2, "dgamma")
    _close(beta_g.grad, beta.grad, 0.5, 2e-2, "dbeta")


def _attn_case(B, H, Sq, Sk, mode, cross, kp):
    torch.manual_seed(1)
    hd = 64
    if cross:
        q = torch.randn(B, Sq, H * hd).bfloat16()
        kv = torch.randn(B, Sk, 2 * H * hd).bfloat16()
        kpad = None
        if kp:
            kpad = torch.zeros(B, Sk, dtype=torch.bool)
            kpad[0, Sk // 2:] = True
        qg, kvg = q.to(dev).requires_grad_(), kv.to(dev).requires_grad_()
        qc, kvc = q.float().requires_grad_(), kv.float().requires_grad_()
        og = cross_attention(qg, kvg, H, mode, kpad.to(dev) if kpad is not None else None)
        oc = cross_attention(qc, kvc, H, mode, kpad)
        do = torch.randn_like(oc).bfloat16()
        og.backward(do.to(dev))
        oc.backward(do.float())
        _close(og, oc, 2e-2, 2e-2, f"attn fwd {mode}")
        _close(qg.grad, qc.grad, 3e-2, 3e-2, "dq")
        _close(kvg.grad, kvc.grad, 3e-2, 3e-2, "dkv")
    else:
        qkv = torch.randn(B, Sq, 3 * H * hd).bfloat16()
        qg = qkv.to(dev).requires_grad_()
        qc = qkv.float().requires_grad_()
        og = self_attention(qg, H, mode)
        oc = self_attention(qc, H, mode)
        do = torch.randn_like(oc).bfloat16()
        og.backward(do.to(dev))
        oc.backward(do.float())
        _close(og, oc, 2e-2, 2e-2, f"attn fwd {mode}")
        _close(qg.grad, qc.grad, 3e-2, 3e-2, f"dqkv {mode}")


@pytest.fixture(params=[1, 0], ids=["single_pass_bwd", "dq_dkdv_pair"])
def bwd_path(request):
    """Attention backward at Sk <= 256: the single-pass 8-wave kernel (default) or the dQ + dK/dV
    kernel pair (C.attn_bwd1(0)); past 256 keys the pair always runs."""
    C = _native.C()
    prev = C.attn_bwd1(-1)
    C.attn_bwd1(request.param)
    yield request.param
    C.attn_bwd1(prev)


@pytest.mark.parametrize("mode", ["none", "reference", "causal"])
@pytest.mark.parametrize("S", [256, 200, 37, 300])
def test_self_attention(bwd_path, mode, S):
    _attn_case(2, 4, S, S, mode, False, False)


@pytest.mark.parametrize("mode", ["none", "reference"])
@pytest.mark.parametrize("kp", [False, True])
def test_cross_attention(bwd_path, mode, kp):
    _attn_case(2, 3, 130, 130 if mode == "reference" else 77, mode, True, kp)


@pytest.mark.parametrize("cross", [False, True])
def test_attention_bwd_single_pass_repeatable(cross):
    """The single-pass backward sums every dQ tile over the key images in a fixed order (no
    atomics): two runs are bitwise equal; Sq (300) > Sk exercises the streamed query chunks."""
    torch.manual_seed(3)
    B, H, hd = 2, 3, 64
    if cross:
        ins = (torch.randn(B, 300, H * hd, device=dev).bfloat16(), torch.randn(B, 250, 2 * H * hd, device=dev).bfloat16())
    else:
        ins = (torch.randn(B, 256, 3 * H * hd, device=dev).bfloat16(),)
    do = torch.randn(B, ins[0].shape[1], H * hd, device=dev).bfloat16()
    outs = []
    for _ in range(2):
        xs = [t.clone().requires_grad_() for t in ins]
        o = cross_attention(xs[0], xs[1], H, "reference") if cross else self_attention(xs[0], H, "reference")
        o.backward(do)
        outs.append([t.grad.clone() for t in xs])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_cross_entropy(dtype):
    torch.manual_seed(2)
    M, V = 777, 10000
    x = torch.randn(M, V).to(dtype)
    lab = torch.randint(0, V, (M,))
    lab[:50] = 0
    xg = x.to(dev).requires_grad_()
    xc = x.float().requires_grad_()
    lg = cross_entropy(xg, lab.to(dev), ignore_index=0)
    lc = cross_entropy(xc, lab, ignore_index=0)
    ref = torch.nn.functional.cross_entropy(x.float(), lab, ignore_index=0)
    _close(lg, ref, 1e-3, 1e-3, "ce loss")
    _close(lc, ref, 1e-5, 1e-5, "ce loss ref")
    lg.backward()
    lc.backward()
    _close(xg.grad, xc.grad, 1e-5, 2e-2, "ce grad")


def test_embedding():
    torch.manual_seed(3)
    V, D, B, S = 1000, 512, 4, 64
    w = torch.nn.Parameter(torch.randn(V, D))
    wg = torch.nn.Parameter(w.detach().to(dev))
    ids = torch.randint(0, V, (B, S))
    ids[0, :5] = 7
    pe = sinusoid_table(S, D)
    rg, rc = R.DropoutRNG(3).to(dev), R.DropoutRNG(3)
    og = embedding(ids.to(dev), wg, pe.to(dev), 0.1, rg, 99, padding_idx=7)
    oc = embedding(ids, w, pe, 0.1, rc, 99, padding_idx=7)
    _close(og, oc, 2e-2, 1e-2, "emb fwd")
    do = torch.randn(B, S, D).bfloat16()
    og.backward(do.to(dev))
    oc.backward(do.float())
    _close(wg.grad, w.grad, 2e-2, 2e-2, "emb grad")
    assert float(wg.grad[7].abs().sum()) == 0.0


@pytest.mark.parametrize("n_tok", [8192, 20000])
def test_embedding_backward_deterministic(n_tok):
    """Id-bucketed, position-ordered backward: bit-reproducible and equal to the fp64 index_add
    reference up to fp32 rounding, also with a 600-token run of one id."""
    torch.manual_seed(4)
    V, D = 300, 512  # few ids -> long runs of repeated ids
    ids = torch.randint(0, V, (n_tok,))
    ids[:600] = 11  # a long run (the padding-tail shape)
    w = torch.nn.Parameter(torch.randn(V, D, device=dev, dtype=torch.float32))
    do = torch.randn(n_tok, D, device=dev)
    grads = []
    for _ in range(2):
        w.grad = None
        out = embedding(ids.to(dev), w, None, 0.0, R.DropoutRNG(1).to(dev), 5, padding_idx=None,
                        out_dtype=torch.float32)
        out.backward(do)
        grads.append(w.grad.clone())
    ref = torch.zeros(V, D, dtype=torch.float64).index_add_(0, ids, do.cpu().double())
    _close(grads[0], ref, 1e-4, 1e-5, "emb grad")
    assert torch.equal(grads[0], grads[1])
    # the id ordering made in the backward (plan-ahead off) instead of beside the forward: same bits
    import importlib
    E = importlib.import_module("sparkmi.ops.embedding")
    prev, E.PLAN_AHEAD = E.PLAN_AHEAD, False
    try:
        w.grad = None
        out = embedding(ids.to(dev), w, None, 0.0, R.DropoutRNG(1).to(dev), 5, padding_idx=None,
                        out_dtype=torch.float32)
        out.backward(do)
    finally:
        E.PLAN_AHEAD = prev
    assert torch.equal(grads[0], w.grad)


@pytest.mark.parametrize("D", [512, 96])
def test_embedding_backward_heavy_buckets(D):
    """Padded-batch shape: ~95 % of the tokens are one id (split over EMB_SPLIT segment
    workgroups + ordered combine), a second heavy id, a light tail; bf16 dout, dropout."""
    torch.manual_seed(5)
    V, T = 10000, 8192
    ids = torch.randint(0, V, (T,))
    ids[torch.randperm(T)[:7700]] = 1
    ids[torch.randperm(T)[:1200]] = 10001 % V  # same bucket family as id 1 for small NB, other slot
    w = torch.nn.Parameter(torch.zeros(V, D, device=dev))
    do = torch.randn(T, D, device=dev).bfloat16()
    grads = []
    for _ in range(2):
        w.grad = None
        out = embedding(ids.to(dev), w, None, 0.1, R.DropoutRNG(2).to(dev), 9, padding_idx=None,
                        out_dtype=torch.bfloat16)
        out.backward(do)
        grads.append(w.grad.clone())
    assert torch.equal(grads[0], grads[1])
    wc = torch.nn.Parameter(torch.zeros(V, D))
    oc = embedding(ids, wc, None, 0.1, R.DropoutRNG(2), 9, padding_idx=None, out_dtype=torch.float32)
    oc.backward(do.float().cpu())
    _close(grads[0], wc.grad, 1e-3, 1e-4, "emb heavy grad")


@pytest.mark.parametrize("act,p", [(None, 0.0), ("relu", 0.1), ("relu", 0.0)])
def test_linear(act, p):
    torch.manual_seed(4)
    M, K, N = 512, 256, 384
    lin = torch.nn.Linear(K, N)
    with torch.no_grad():  # the GPU computes with the bf16 weight shadow: give the reference the same weights
        lin.weight.copy_(lin.weight.bfloat16().float())
        lin.bias.copy_(lin.bias.bfloat16().float())
    wg = torch.nn.Parameter(lin.weight.detach().to(dev))
    bg = torch.nn.Parameter(lin.bias.detach().to(dev))
    x = torch.randn(M, K).bfloat16()
    xg = x.to(dev).requires_grad_()
    xc = x.float().requires_grad_()
    rg, rc = R.DropoutRNG(5).to(dev), R.DropoutRNG(5)
    yg = linear(xg, wg, bg, act, p, rg, 11)
    yc = linear(xc, lin.weight, lin.bias, act, p, rc, 11)
    _close(yg, yc, 5e-2, 2e-2, "linear fwd")
    dy = torch.randn(M, N).bfloat16()
    yg.backward(dy.to(dev))
    yc.backward(dy.float())
    _close(xg.grad, xc.grad, 5e-2, 3e-2, "dx")
    _close(wg.grad, lin.weight.grad, 0.5, 3e-2, "dw")
    _close(bg.grad, lin.bias.grad, 0.5, 3e-2, "db")


def test_adam_sgd_flat():
    from sparkmi.optim import SGD, Adam
    from sparkmi.utils.flat import FlatParams
    torch.manual_seed(5)
    for Opt, kw in ((Adam, dict(lr=1e-2, weight_decay=0.01)), (SGD, dict(lr=0.1, momentum=0.9))):
        mc = torch.nn.Sequential(torch.nn.Linear(33, 17), torch.nn.Linear(17, 5))
        mg = torch.nn.Sequential(torch.nn.Linear(33, 17), torch.nn.Linear(17, 5)).to(dev)
        mg.load_state_dict(mc.state_dict())
        fc, fg = FlatParams(mc), FlatParams(mg)
        oc, og = Opt(fc, **kw), Opt(fg, **kw)
        for _ in range(3):
            g = torch.randn(fc.numel)
            fc.grad.copy_(g)
            fg.grad.copy_(g.to(dev))
            oc.step()
            og.step()
        _close(fg.master, fc.master, 1e-5, 1e-5, Opt.__name__)
        _close(fg.shadow, fg.master, 1e-2, 1e-2, "shadow")
        assert float(og.step_t.item()) == 3.0


def test_optimizer_step_counter_many_blocks_graph():
    """The update kernels advance the device step counter themselves (last block's ticket):
    check it with a multi-thousand-block grid, eagerly and inside a replayed HIP graph, against
    torch.optim.Adam (bias corrections depend on the count)."""
    from sparkmi.optim import Adam
    from sparkmi.utils.flat import FlatParams
    torch.manual_seed(6)
    mc = torch.nn.Linear(2048, 1024)
    mg = torch.nn.Linear(2048, 1024).to(dev)
    mg.load_state_dict(mc.state_dict())
    fg = FlatParams(mg)
    og = Adam(fg, lr=1e-3)
    ref = torch.optim.Adam(mc.parameters(), lr=1e-3)
    grads = [torch.randn(fg.numel) for _ in range(6)]

    pairs = list(zip(mc.parameters(), mg.parameters()))

    def ref_step(g):  # the flat layout is padded and in reverse order: map through param_range
        for pc, pg in pairs:
            a, b = fg.param_range(pg)
            pc.grad = g[a:b].view_as(pc).clone()
        ref.step()

    for g in grads[:2]:
        fg.grad.copy_(g.to(dev))
        og.step()
        ref_step(g)
    static_g = torch.empty(fg.numel, device=dev)
    graph = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(graph):
        fg.grad.copy_(static_g)
        og.step()
    for g in grads[2:]:
        static_g.copy_(g.to(dev))
        graph.replay()
        ref_step(g)
    torch.cuda.synchronize()
    assert float(og.step_t.item()) == 6.0
    for pc, pg in pairs:
        a, b = fg.param_range(pg)
        _close(fg.master[a:b].cpu(), pc.detach().reshape(-1), 1e-5, 1e-5, "adam graph")


def test_transformer_gpu_vs_cpu():
    import os
    from safetensors.torch import load_file
    from sparkmi.models.transformer import Transformer
    from sparkmi.utils.flat import FlatParams
    gold = load_file(os.path.join(os.path.dirname(__file__), "fixtures", "transformer_ref.safetensors"))
    sd = {k[len("param."):]: v for k, v in gold.items() if k.startswith("param.")}
    m = Transformer(d_model=128, ffn_hidden=256, num_heads=2, num_layers=2, max_sequence_length=16,
                    src_vocab_size=50, tgt_vocab_size=60)
    m.load_state_dict(sd)
    m = m.to(dev).eval()
    FlatParams(m)
    from sparkmi.models.transformer import create_look_ahead_mask
    la = create_look_ahead_mask(gold["tgt"].shape[1])
    logits = m(gold["src"].to(dev), gold["tgt"].to(dev), None, la, la)
    _close(logits, gold["logits"], 0.15, 0.05, "logits")
    loss = m.loss(logits, gold["tgt"].to(dev))
    _close(loss.reshape(1), gold["loss"], 2e-2, 2e-2, "loss")
    loss.backward()
    for name, p in m.named_parameters():
        g = gold["grad." + name]
        rel = (p.grad.cpu() - g).norm() / (g.norm() + 1e-6)
        assert rel < 0.1, (name, float(rel))


def test_ffn_fused():
    from sparkmi.ops.linear import ffn
    torch.manual_seed(6)
    M, D, H = 1024, 512, 1024
    l1, l2 = torch.nn.Linear(D, H), torch.nn.Linear(H, D)
    with torch.no_grad():
        for l in (l1, l2):
            l.weight.copy_(l.weight.bfloat16().float())
    g1, g2 = torch.nn.Linear(D, H).to(dev), torch.nn.Linear(H, D).to(dev)
    g1.load_state_dict(l1.state_dict())
    g2.load_state_dict(l2.state_dict())
    x = torch.randn(M, D).bfloat16()
    xg = x.to(dev).requires_grad_()
    xc = x.float().requires_grad_()
    rg, rc = R.DropoutRNG(8).to(dev), R.DropoutRNG(8)
    yg = ffn(xg, g1, g2, 0.1, rg, 77)
    yc = ffn(xc, l1, l2, 0.1, rc, 77)
    _close(yg, yc, 6e-2, 3e-2, "ffn fwd")
    dy = torch.randn(M, D).bfloat16()
    yg.backward(dy.to(dev))
    yc.backward(dy.float())
    _close(xg.grad, xc.grad, 6e-2, 3e-2, "ffn dx")
    for a, b, n in ((g1.weight, l1.weight, "w1"), (g2.weight, l2.weight, "w2"), (g1.bias, l1.bias, "b1"),
                    (g2.bias, l2.bias, "b2")):
        rel = (a.grad.cpu() - b.grad).norm() / b.grad.norm()
        assert rel < 2e-2, (n, float(rel))


@pytest.mark.parametrize("T,V,D,pad", [(4128, 95812, 32, 0), (8192, 10000, 512, 3), (8192, 50, 96, None)])
def test_embedding_backward_pair_vs_bucketed(T, V, D, pad):
    """The 3-launch pair-compare backward (<= 8192 tokens: the LSTM's 32 x 129 and the
    transformer's 32 x 256 batches) against the bucketed-list one: equal to fp32 rounding, both
    bit-reproducible, padding rows untouched; V = 50: groups of ~160 tokens (5 chunks each)."""
    torch.manual_seed(6)
    C = _native.C()
    ids = torch.randint(0, V, (T,))
    ids[: T // 4] = pad if pad is not None else 1
    do = torch.randn(T, D, device=dev)
    prev, prev_max = C.emb_pair(-1), C.emb_pair_max(-1)
    C.emb_pair_max(8192)
    out = {}
    try:
        for algo in (1, 0):
            C.emb_pair(algo)
            gs = []
            for _ in range(2):
                w = torch.nn.Parameter(torch.zeros(V, D, device=dev))
                o = embedding(ids.to(dev), w, None, 0.1, R.DropoutRNG(2).to(dev), 9, padding_idx=pad,
                              out_dtype=torch.float32)
                o.backward(do)
                gs.append(w.grad.clone())
            assert torch.equal(gs[0], gs[1]), algo
            out[algo] = gs[0]
    finally:
        C.emb_pair(prev)
        C.emb_pair_max(prev_max)
    _close(out[1], out[0], 1e-5, 1e-5, "pair vs bucketed")
    if pad is not None:
        assert float(out[1][pad].abs().sum()) == 0.0
