"""StepRunner(bind_inputs=True): one graph per HBM-resident batch, read in place — same losses and
parameters as the copying graph path (GPU), and a plain eager fallback on CPU."""
import pytest
import torch

from sparkmi.models.mlp import MultilayerPerceptron
from sparkmi.optim import SGD
from sparkmi.train.runner import StepRunner
from sparkmi.utils.flat import FlatParams


def _run(device, bind, batches, steps):
    torch.manual_seed(0)
    model = MultilayerPerceptron((4, 5, 4, 3)).to(device).train()
    flat = FlatParams(model, shadow=False)
    opt = SGD(flat, lr=0.05)
    r = StepRunner(model, lambda m, x, y: m.loss(x, y), opt, graph=device == "cuda", warmup_eager=2, bind_inputs=bind)
    losses = [float(r.step(*batches[i % len(batches)])) for i in range(steps)]
    return losses, [p.detach().cpu().clone() for p in model.parameters()], r


def _batches(device):
    g = torch.Generator().manual_seed(3)
    return [(torch.rand(30, 4, generator=g).to(device), torch.randint(0, 3, (30,), generator=g).to(device))
            for _ in range(3)]


def test_bind_inputs_cpu_is_eager():
    b = _batches("cpu")
    l0, p0, _ = _run("cpu", False, b, 6)
    l1, p1, r = _run("cpu", True, b, 6)
    assert l0 == l1 and all(torch.equal(a, c) for a, c in zip(p0, p1))
    assert not r._bound


@pytest.mark.gpu
def test_bind_inputs_matches_copying_graph():
    b = _batches("cuda")
    l0, p0, _ = _run("cuda", False, b, 10)
    l1, p1, r = _run("cuda", True, b, 10)
    assert len(r._bound) == len(b)  # one graph per batch, each read in place
    assert l0 == l1
    assert all(torch.equal(a, c) for a, c in zip(p0, p1))


@pytest.mark.gpu
def test_multi_step_graph_matches_single_steps():
    """run_steps with unroll: each cycle over the batches replays as ONE graph of that many
    steps — the same losses and parameters as one graph per step."""
    b = _batches("cuda")

    def go(unroll):
        torch.manual_seed(0)
        model = MultilayerPerceptron((4, 5, 4, 3)).cuda().train()
        flat = FlatParams(model, shadow=False)
        r = StepRunner(model, lambda m, x, y: m.loss(x, y), SGD(flat, lr=0.05), graph=True, warmup_eager=2,
                       bind_inputs=True)
        r.unroll = unroll
        for i in range(4):
            r.step(*b[i % 3])
        loss = r.run_steps([b[i % 3] for i in range(3 * 3 + 2)])
        return float(loss), [p.detach().cpu().clone() for p in model.parameters()], r

    l1, p1, _ = go(1)
    l3, p3, r3 = go(3)
    assert len(r3._multi) == 1
    assert l1 == l3 and all(torch.equal(a, c) for a, c in zip(p1, p3))
