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
