"""CNN: module/state_dict parity with the reference FashionMNISTModel layout (CPU), and the fused
whole-network HIP kernel (forward, loss, every parameter gradient) against the fp32 torch
reference (GPU)."""
import pytest
import torch

from sparkmi.models.cnn import FashionMNISTModel
from sparkmi.ops.cnn import reference_logits


def _torch_ref_model():
    import torch.nn as nn
    return nn.ModuleDict()


def test_param_count_and_names():
    m = FashionMNISTModel(1, 10, 10)
    assert sum(p.numel() for p in m.parameters()) == 7740
    keys = set(m.state_dict().keys())
    assert "block_1.0.weight" in keys and "block_2.2.bias" in keys and "classifier.1.weight" in keys


def test_cpu_loss_grad_matches_autograd():
    torch.manual_seed(0)
    m = FashionMNISTModel()
    x = torch.rand(4, 1, 28, 28)
    y = torch.randint(0, 10, (4,))
    loss = m.loss(x, y)
    loss.backward()
    ref = torch.nn.functional.cross_entropy(reference_logits(x, [p.detach().requires_grad_() for p in m.param_list()]),
                                            y)
    assert abs(float(loss) - float(ref)) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("u8", [False, True])
def test_fused_cnn_kernel_vs_torch(u8):
    torch.manual_seed(1)
    B = 32
    mc = FashionMNISTModel()
    mg = FashionMNISTModel().cuda()
    mg.load_state_dict(mc.state_dict())
    if u8:
        x = torch.randint(0, 256, (B, 1, 28, 28), dtype=torch.uint8)
    else:
        x = torch.rand(B, 1, 28, 28)
    y = torch.randint(0, 10, (B,))
    lg = mg.loss(x.cuda(), y.cuda())
    lc = mc.loss(x, y)
    assert abs(float(lg) - float(lc)) < 1e-4, (float(lg), float(lc))
    lg.backward()
    lc.backward()
    for (n, pg), pc in zip(mg.named_parameters(), mc.parameters()):
        rel = float((pg.grad.cpu() - pc.grad).norm() / (pc.grad.norm() + 1e-12))
        assert rel < 1e-4, (n, rel)
    zg = mg(x.cuda())
    zc = mc(x)
    assert float((zg.cpu() - zc).abs().max()) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("cin,hidden", [(1, 12), (2, 8), (3, 12), (1, 13), (1, 4)])
def test_fused_cnn_kernel_channel_counts(cin, hidden):
    """Clamped-group kernel instance (C != 10; C = 13 is the LDS-residency maximum).  Inputs are
    random floats: a config whose CPU/GPU activations land on a max-pool near-tie (1e-7 apart)
    routes that window's gradient to the neighbour (bias grads equal, weight grads ~1e-3 off),
    e.g. (3, 8) at this seed — a tie-break artefact, not a kernel error. instances vs the CPU reference."""
    torch.manual_seed(2)
    B = 8
    mc = FashionMNISTModel(cin, hidden, 10)
    mg = FashionMNISTModel(cin, hidden, 10).cuda()
    mg.load_state_dict(mc.state_dict())
    x = torch.rand(B, cin, 28, 28)
    y = torch.randint(0, 10, (B,))
    lg = mg.loss(x.cuda(), y.cuda())
    lc = mc.loss(x, y)
    assert abs(float(lg) - float(lc)) < 1e-4, (float(lg), float(lc))
    lg.backward()
    lc.backward()
    for (n, pg), pc in zip(mg.named_parameters(), mc.parameters()):
        rel = float((pg.grad.cpu() - pc.grad).norm() / (pc.grad.norm() + 1e-12))
        assert rel < 1e-4, (n, rel)


def _bf16_ref_logits(x, params):
    """fp32 CNN with every convolution's operands rounded to bf16 (what the matrix-core path
    multiplies; products and sums in fp32)."""
    import torch.nn.functional as F
    r = lambda t: t.bfloat16().float()  # noqa: E731
    w1, b1, w2, b2, w3, b3, w4, b4, wf, bf = params
    h = x.float() / 255.0 if x.dtype == torch.uint8 else x.float()
    h = F.relu(F.conv2d(r(h), r(w1), b1, padding=1))
    h = F.relu(F.conv2d(r(h), r(w2), b2, padding=1))
    h = F.max_pool2d(h, 2)
    h = F.relu(F.conv2d(r(h), r(w3), b3, padding=1))
    h = F.relu(F.conv2d(r(h), r(w4), b4, padding=1))
    h = F.max_pool2d(h, 2)
    return F.linear(h.flatten(1), wf, bf)


@pytest.mark.gpu
def test_fused_cnn_bf16_mfma_vs_reference():
    """bf16 matrix-core convolutions: forward equals the bf16-operand fp32 reference to fp32
    summation error; gradients follow the fp32 reference to bf16 precision."""
    torch.manual_seed(3)
    B = 32
    mc = FashionMNISTModel()
    mg = FashionMNISTModel(dtype="bf16").cuda()
    mg.load_state_dict(mc.state_dict())
    x = torch.rand(B, 1, 28, 28)
    y = torch.randint(0, 10, (B,))
    zg = mg(x.cuda()).cpu()
    zr = _bf16_ref_logits(x, [p.detach() for p in mc.param_list()])
    assert float((zg - zr).abs().max()) < 2e-3, float((zg - zr).abs().max())
    lg = mg.loss(x.cuda(), y.cuda())
    lc = mc.loss(x, y)
    assert abs(float(lg) - float(lc)) < 2e-2, (float(lg), float(lc))
    lg.backward()
    lc.backward()
    # bf16 operands in three chained dgrads: the first conv's weight gradient (a sum over
    # 25k cancelling terms) is ~10 % off the fp32 one, the later layers ~1-3 %
    for (n, pg), pc in zip(mg.named_parameters(), mc.parameters()):
        a, b = pg.grad.cpu().flatten(), pc.grad.flatten()
        rel = float((a - b).norm() / (b.norm() + 1e-12))
        cos = float(torch.nn.functional.cosine_similarity(a, b, dim=0))
        assert rel < 0.15 and cos > 0.99, (n, rel, cos)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_fused_cnn_gradients_bit_reproducible(dtype):
    """Per-image slabs + fixed-order reductions (no float atomics): identical backwards give
    bit-identical gradients."""
    torch.manual_seed(4)
    m = FashionMNISTModel(dtype=dtype).cuda()
    x = torch.rand(32, 1, 28, 28, device="cuda")
    y = torch.randint(0, 10, (32,), device="cuda")
    out = []
    for _ in range(2):
        for p in m.parameters():
            p.grad = None
        m.loss(x, y).backward()
        out.append([p.grad.clone() for p in m.parameters()])
    for a, b in zip(*out):
        assert torch.equal(a, b)


CNN_MAXB = 64  # csrc/include/smi_cnn.h


def test_cnn_fused_batch_limit_is_cnn_maxb():
    """The fused step takes every batch up to CNN_MAXB for the reference model in both dtypes (the
    fused tail's LDS is part of the kernel's allocation, checked per dtype: csrc/kernels/cnn.hip
    smi_cnn_fused_ok) and none past it; the Python model reports the same limit."""
    from sparkmi import _native
    if not _native.has_native():
        pytest.skip("native library not built")
    C = _native.C()
    for bf in (0, 1):
        assert C.cnn_max_batch(10, 1, 10, bf) == CNN_MAXB
        assert all(C.cnn_fused_ok(10, 1, 10, b, bf) for b in (1, 20, 32, 59, 63, CNN_MAXB))
        assert not C.cnn_fused_ok(10, 1, 10, CNN_MAXB + 1, bf) and not C.cnn_fused_ok(10, 1, 10, 0, bf)
    assert FashionMNISTModel(1, 10, 10).fused_batch_limit() == CNN_MAXB


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,B", [("fp32", 32), ("bf16", 32), ("fp32", 20), ("bf16", CNN_MAXB),
                                     ("fp32", CNN_MAXB)])
def test_fused_sgd_step_matches_unfused(dtype, B):
    """The one-launch CNN step (fused slab reduction + SGD in the kernel's ticketed tail) follows
    the three-launch path (kernel -> batch gradient reduce -> SGD kernel) step for step, keeps the
    bf16 shadow in sync, is bit-reproducible, and replays identically inside a HIP graph
    (StepRunner's single-executor fused_step path).  B = 20: a ragged last group of images;
    B = CNN_MAXB: the limit itself, 320 workgroups with the weight-gradient helpers — more than the CUs."""
    from sparkmi.optim import SGD
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    g = torch.Generator().manual_seed(3)
    xs = (torch.rand(6, B, 1, 28, 28, generator=g) * 255).to(torch.uint8).cuda()
    ys = torch.randint(0, 10, (6, B), generator=g).cuda()

    def run(mode):
        torch.manual_seed(0)
        m = FashionMNISTModel(1, 10, 10, dtype=dtype).cuda().train()
        flat = FlatParams(m, shadow=True)
        opt = SGD(flat, lr=0.05)
        losses = []
        if mode == "graph":
            r = StepRunner(m, lambda mm, x, y: mm.loss(x, y), opt, graph=True, warmup_eager=2,
                           fused_step=lambda mm, o, x, y: mm.fused_sgd_step(o, x, y))
        for i in range(6):
            if mode == "fused":
                loss = m.fused_sgd_step(opt, xs[i], ys[i])
                assert loss is not None
            elif mode == "graph":
                loss = r.step(xs[i], ys[i])
            else:
                loss = m.loss(xs[i], ys[i])
                loss.backward()
                opt.step()
            losses.append(float(loss))
        torch.cuda.synchronize()
        return losses, flat.master.clone(), flat.shadow.clone(), float(opt.step_t.item())

    lf, pf, sf, tf = run("fused")
    lf2, pf2, _, _ = run("fused")
    lg, pg, _, _ = run("graph")
    lu, pu, _, tu = run("unfused")
    assert lf == lf2 and torch.equal(pf, pf2)           # deterministic
    assert lg == lf and torch.equal(pg, pf)             # graph replay == eager fused
    assert torch.equal(sf, pf.to(torch.bfloat16))       # shadow refreshed
    assert tf == tu == 6.0                              # step counter advanced per step
    for a, b in zip(lf, lu):
        assert abs(a - b) <= 1e-5 * abs(b) + 1e-6, (lf, lu)
    torch.testing.assert_close(pf, pu, rtol=1e-5, atol=5e-6)  # fp32 sums in another order


@pytest.mark.gpu
def test_fused_step_past_the_limit_warns_and_falls_back():
    """A batch past CNN_MAXB runs the multi-launch step (None from the fused step) and says so once."""
    from sparkmi.optim import SGD
    from sparkmi.utils.flat import FlatParams
    m = FashionMNISTModel(1, 10, 10, dtype="bf16").cuda().train()
    opt = SGD(FlatParams(m, shadow=True), lr=0.05)
    x = torch.rand(CNN_MAXB + 1, 1, 28, 28, device="cuda")
    y = torch.randint(0, 10, (CNN_MAXB + 1,), device="cuda")
    with pytest.warns(RuntimeWarning, match="exceeds the fused step's limit"):
        assert m.fused_sgd_step(opt, x, y) is None
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        assert m.fused_sgd_step(opt, x, y) is None  # once per model
