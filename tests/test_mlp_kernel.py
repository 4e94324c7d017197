"""Fused MLP kernels (csrc/kernels/mlp.hip): loss and every parameter gradient against the fp32
torch reference of the same network, on the GPU (batch 30 = the reference minibatch; 200 and
5000 rows = several 64-row chunks / blocks; sigmoid and relu; MLlib-style row weights)."""
import pytest
import torch

from sparkmi.models.mlp import MultilayerPerceptron


def _torch_loss(m, x, y, act, row_weight=None):
    h = x
    lins = m.linears()
    for i, lin in enumerate(lins):
        h = h @ lin.weight.t() + lin.bias
        if i < len(lins) - 1:
            h = torch.sigmoid(h) if act == "sigmoid" else torch.relu(h)
    rl = torch.logsumexp(h, 1) - h.gather(1, y[:, None]).squeeze(1)
    w = row_weight if row_weight is not None else torch.full_like(rl, 1.0 / x.shape[0])
    return (rl * w).sum()


@pytest.mark.gpu
@pytest.mark.parametrize("n,layers,act,weighted", [(30, (4, 5, 4, 3), "sigmoid", False),
                                                   (200, (4, 5, 4, 3), "relu", False),
                                                   (5000, (8, 32, 16, 5), "sigmoid", True)])
def test_mlp_kernel_vs_torch(n, layers, act, weighted):
    torch.manual_seed(0)
    mc = MultilayerPerceptron(layers, activation=act)
    mg = MultilayerPerceptron(layers, activation=act).cuda()
    mg.load_state_dict(mc.state_dict())
    x = torch.rand(n, layers[0]) * 2 - 1
    y = torch.randint(0, layers[-1], (n,))
    rw = torch.rand(n) / n if weighted else None
    lg = mg.loss(x.cuda(), y.cuda(), None if rw is None else rw.cuda())
    lc = _torch_loss(mc, x, y, act, rw)
    assert abs(float(lg) - float(lc)) < 1e-5 * max(1.0, abs(float(lc))), (float(lg), float(lc))
    lg.backward()
    lc.backward()
    for (name, pg), pc in zip(mg.named_parameters(), mc.parameters()):
        rel = float((pg.grad.cpu() - pc.grad).norm() / (pc.grad.norm() + 1e-12))
        assert rel < 1e-4, (name, rel)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [30, 5000])
def test_mlp_gradients_bit_reproducible(n):
    """Cross-block sums are a block-order reduction, not float atomics: the same backward twice
    gives bit-identical gradients (5000 rows = 79 blocks)."""
    torch.manual_seed(1)
    m = MultilayerPerceptron((8, 32, 16, 5)).cuda()
    x = (torch.rand(n, 8) * 2 - 1).cuda()
    y = torch.randint(0, 5, (n,)).cuda()
    grads = []
    for _ in range(2):
        for p in m.parameters():
            p.grad = None
        m.loss(x, y).backward()
        grads.append([p.grad.clone() for p in m.parameters()])
    for a, b in zip(*grads):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [30, 700])
def test_mlp_fused_sgd_step_equals_chain(n):
    """ONE launch (forward + CE + backward + SGD) == loss kernel + backward kernel + SGD kernel."""
    from sparkmi.optim import SGD
    from sparkmi.utils.flat import FlatParams
    torch.manual_seed(2)
    a = MultilayerPerceptron((4, 5, 4, 3)).cuda()
    b = MultilayerPerceptron((4, 5, 4, 3)).cuda()
    b.load_state_dict(a.state_dict())
    fa, fb = FlatParams(a, shadow=False), FlatParams(b, shadow=False)
    oa, ob = SGD(fa, lr=0.05), SGD(fb, lr=0.05)
    g = torch.Generator().manual_seed(3)
    for _ in range(5):
        x = (torch.rand(n, 4, generator=g) * 2 - 1).cuda()
        y = torch.randint(0, 3, (n,), generator=g).cuda()
        la = a.fused_sgd_step(oa, x, y)
        assert la is not None
        lb = b.loss(x, y)
        lb.backward()
        ob.step()
        assert abs(float(la) - float(lb)) <= 1e-6 * abs(float(lb)), (float(la), float(lb))
    torch.testing.assert_close(fa.master, fb.master, atol=1e-6, rtol=1e-6)
    assert float(oa.step_t) == float(ob.step_t) == 5.0
    assert torch.count_nonzero(fa.grad) == 0  # the fused step never materialises gradients


@pytest.mark.gpu
@pytest.mark.parametrize("n,act,weighted", [(30, "sigmoid", False), (64, "relu", True), (1, "sigmoid", False)])
def test_mlp_small_kernel_matches_generic(n, act, weighted):
    """The compile-time 4-5-4-3 kernel (registers, one wave; csrc/kernels/mlp.hip mlp_small_kernel)
    against the generic kernel: loss, gradients (mode 1) and the fused SGD step (mode 2)."""
    from sparkmi import _native
    from sparkmi.ops.mlp import mlp_sgd_step
    C = _native.C()
    torch.manual_seed(3)
    x = (torch.rand(n, 4) * 2 - 1).cuda()
    y = torch.randint(0, 3, (n,)).cuda()
    rw = (torch.rand(n) / n).cuda() if weighted else None
    base = MultilayerPerceptron((4, 5, 4, 3), activation=act).cuda()
    out = {}
    prev = C.mlp_small(-1)
    try:
        for small in (1, 0):
            C.mlp_small(small)
            m = MultilayerPerceptron((4, 5, 4, 3), activation=act).cuda()
            m.load_state_dict(base.state_dict())
            loss = m.loss(x, y, rw)
            loss.backward()
            grads = [p.grad.clone() for p in m.parameters()]
            lins = m.linears()
            lr = torch.tensor([0.1], device="cuda")
            step = torch.zeros(1, device="cuda")
            l2 = mlp_sgd_step(x, y, [l.weight for l in lins], [l.bias for l in lins], lr, step, act, rw)
            out[small] = (loss.detach(), grads, l2, [p.detach().clone() for p in m.parameters()], step.clone())
    finally:
        C.mlp_small(prev)
    a, b = out[1], out[0]
    torch.testing.assert_close(a[0], b[0], rtol=1e-6, atol=1e-7)
    for ga, gb in zip(a[1], b[1]):
        torch.testing.assert_close(ga, gb, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(a[2], b[2], rtol=1e-6, atol=1e-7)
    for pa, pb in zip(a[3], b[3]):
        torch.testing.assert_close(pa, pb, rtol=1e-6, atol=1e-7)
    assert float(a[4]) == float(b[4]) == 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("steps,n", [(8, 30), (1, 64), (32, 7)])
def test_mlp_multi_step_kernel_bitwise_equals_single_steps(steps, n):
    """``steps`` fused SGD steps in ONE launch (parameters on chip between the steps,
    csrc/kernels/mlp.hip mlp_small_steps_kernel) == the same steps as one launch each: bitwise
    parameters, per-step losses and the step counter."""
    from sparkmi.optim import SGD
    from sparkmi.utils.flat import FlatParams
    torch.manual_seed(4)
    a = MultilayerPerceptron((4, 5, 4, 3)).cuda()
    b = MultilayerPerceptron((4, 5, 4, 3)).cuda()
    b.load_state_dict(a.state_dict())
    fa, fb = FlatParams(a, shadow=False), FlatParams(b, shadow=False)
    oa, ob = SGD(fa, lr=0.3), SGD(fb, lr=0.3)
    g = torch.Generator().manual_seed(5)
    batches = [((torch.rand(n, 4, generator=g) * 2 - 1).cuda(), torch.randint(0, 3, (n,), generator=g).cuda())
               for _ in range(steps)]
    la = a.fused_sgd_steps(oa, batches)
    assert la is not None and len(la) == steps
    lb = [b.fused_sgd_step(ob, x, y) for x, y in batches]
    assert torch.equal(torch.stack(la), torch.stack(lb))
    assert torch.equal(fa.master, fb.master)
    assert float(oa.step_t) == float(ob.step_t) == float(steps)


@pytest.mark.gpu
@pytest.mark.parametrize("unroll,nb,log_every,steps", [(4, 10, 5, 23), (40, 50, 50, 95)])
def test_mlp_trainer_index_mode_multistep_bitwise(unroll, nb, log_every, steps):
    """The MLP recipe path: Trainer + DeviceLoader(fixed=True) with the multi-step kernel reading
    its shuffled rows from the dataset (index mode, `unroll` steps per graph, an epoch boundary
    inside the run) trains bitwise the same parameters as the per-batch gather with one launch per
    step.  unroll 40 > the kernel's 32 steps per launch: two launches per group."""
    from sparkmi.data.dataset import DeviceLoader
    from sparkmi.optim import SGD
    from sparkmi.recipes.mlp import MLPConfig
    from sparkmi.train.trainer import Trainer

    def run(fixed, unroll):
        torch.manual_seed(0)
        g = torch.Generator().manual_seed(8)
        x = torch.rand(30 * nb, 4, generator=g) * 2 - 1
        y = torch.randint(0, 3, (30 * nb,), generator=g)
        cfg = MLPConfig(batch_size=30, lr=0.2, log_every=log_every, verbose=False, unroll=unroll, max_steps=steps)
        loader = DeviceLoader([x, y], 30, "cuda", shuffle=True, drop_last=True, seed=3, fixed=fixed)
        model = MultilayerPerceptron((4, 5, 4, 3))
        tr = Trainer(model, lambda m, a, b: m.loss(a, b), lambda flat: SGD(flat, lr=cfg.lr), cfg, "cuda", 0, 1, "t",
                     shadow=False, fused_step=lambda m, o, a, b: m.fused_sgd_step(o, a, b),
                     fused_steps=lambda m, o, bs: m.fused_sgd_steps(o, bs))
        res = tr.fit(loader, 10)
        recs = list(tr.metrics.records)
        tr.close()
        return tr.flat.master.cpu().clone(), res, recs, tr.runner

    pa, ra, la, _ = run(False, 1)
    pb, rb, lb, runner = run(True, unroll)
    assert ra["steps"] == rb["steps"] == steps
    assert runner.pre_step is None, "index mode engaged"
    assert runner._multi, "multi-step graphs ran"
    assert torch.equal(pa, pb)
    assert [r["step"] for r in la] == [r["step"] for r in lb]
    for u, v in zip(la, lb):
        assert abs(u["loss"] - v["loss"]) <= 1e-6 * max(1.0, abs(u["loss"])), (u, v)
