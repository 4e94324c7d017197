"""LSTM text classifier (distributed_lstm.py:110-135): reference-layout parity on CPU, fused HIP
kernel (forward + BPTT, inter-layer dropout, padding_idx, h0/c0 grads) vs the fp32 torch
reference on GPU."""
import pytest
import torch

from sparkmi.models.lstm import LSTM
from sparkmi.ops import lstm as LS

REF_KEYS = ["embedding.weight", "lstm.weight_ih_l0", "lstm.weight_hh_l0", "lstm.bias_ih_l0", "lstm.bias_hh_l0",
            "lstm.weight_ih_l1", "lstm.weight_hh_l1", "lstm.bias_ih_l1", "lstm.bias_hh_l1", "fc_out.weight",
            "fc_out.bias"]


def _model(V=50, H=32, L=2, C=4, pad=5, seed=0):
    torch.manual_seed(seed)
    return LSTM(V, H, H, C, num_layers=L, padding_idx=pad)


def test_state_dict_keys_match_reference():
    m = _model()
    assert list(m.state_dict().keys()) == REF_KEYS
    assert m.state_dict()["lstm.weight_ih_l0"].shape == (128, 32)
    assert m.state_dict()["fc_out.weight"].shape == (4, 32)


def test_reference_forward_equals_torch_lstm():
    m = _model().eval()
    ids = torch.randint(0, 50, (3, 11))
    h0, c0 = torch.randn(2, 3, 32), torch.randn(2, 3, 32)
    pred, hn, cn = m(ids, h0, c0)
    out, (h2, c2) = m.lstm(m.embedding(ids), (h0, c0))
    torch.testing.assert_close(pred, m.fc_out(out), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(hn, h2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(cn, c2, rtol=1e-5, atol=1e-5)


def test_training_dropout_and_padding_grad():
    m = _model().train()
    ids = torch.randint(0, 50, (4, 9))
    ids[:, -3:] = 5
    loss, last = m.loss(ids, torch.randint(0, 4, (4,)))
    loss.backward()
    assert m.embedding.weight.grad[5].abs().sum() == 0
    assert last.shape == (4, 4)
    m.eval()
    a, _, _ = m(ids)
    b, _, _ = m(ids)
    torch.testing.assert_close(a, b)


def _grads(m):
    return [p.grad.detach().clone() if p.grad is not None else None for p in m.param_list()]


@pytest.mark.gpu
@pytest.mark.parametrize("L,H,E,p", [(2, 32, 32, 0.5), (1, 32, 32, 0.0), (3, 16, 24, 0.3), (2, 64, 64, 0.0)])
def test_lstm_kernel_matches_reference(L, H, E, p):
    torch.manual_seed(1)
    V, C, B, T, pad = 97, 4, 5, 37, 3
    m = LSTM(V, E, H, C, num_layers=L, padding_idx=pad, dropout=p).cuda()
    if E != H:  # embedding width = hidden in the reference model; exercise E != H through the op directly
        m.embedding = torch.nn.Embedding(V, E, padding_idx=pad).cuda()
    m.train()
    ids = torch.randint(0, V, (B, T), device="cuda")
    ids[0, -5:] = pad
    h0 = torch.randn(L, B, H, device="cuda", requires_grad=True)
    c0 = torch.randn(L, B, H, device="cuda", requires_grad=True)
    params = m.param_list()
    pred, hn, cn = LS.lstm_classifier(ids, h0, c0, params, L, p, True, m.rng, m.salt, pad)
    w = torch.randn_like(pred)
    (pred * w).sum().add_((hn * 0.3).sum()).add_((cn * 0.7).sum()).backward()
    gk = _grads(m)
    dh0k, dc0k = h0.grad.clone(), c0.grad.clone()
    for q in params:
        q.grad = None
    h0.grad = c0.grad = None
    seed = m.rng.current()
    pr, hr, cr = LS.reference_forward(ids, h0, c0, params, L, p, seed, m.salt, pad)
    (pr * w).sum().add_((hr * 0.3).sum()).add_((cr * 0.7).sum()).backward()
    torch.testing.assert_close(pred, pr, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(hn, hr, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(cn, cr, rtol=1e-4, atol=1e-4)
    for a, b in zip(gk, _grads(m)):
        torch.testing.assert_close(a, b, rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(dh0k, h0.grad, rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(dc0k, c0.grad, rtol=2e-3, atol=2e-3)
    assert gk[0][pad].abs().sum() == 0


@pytest.mark.gpu
def test_lstm_gradients_bit_reproducible():
    """Slab + sequence-order reduction for the weights, sorted segment sums for the embedding
    table: two identical backwards give bit-identical gradients (32 sequences, repeated ids)."""
    torch.manual_seed(2)
    V, C, B, T, pad, L, H = 40, 4, 32, 129, 3, 2, 32
    m = LSTM(V, H, H, C, num_layers=L, padding_idx=pad, dropout=0.5).cuda().train()
    ids = torch.randint(0, V, (B, T), device="cuda")
    params = m.param_list()
    out = []
    for _ in range(2):
        for q in params:
            q.grad = None
        pred, hn, cn = LS.lstm_classifier(ids, None, None, params, L, 0.5, True, m.rng, m.salt, pad)
        pred[:, -1].square().sum().backward()
        out.append(_grads(m))
    for a, b in zip(*out):
        assert torch.equal(a, b)
    # the id ordering made by the forward launch's side workgroups (the path above) vs made by the
    # backward itself (meta without the grad-mode flag: no plan): the same bits
    for q in params:
        q.grad = None
    pred, _, _, _ = LS.LSTMFn.apply(ids, None, None, (L, 0.5, m.rng, m.salt, pad), *params)
    pred[:, -1].square().sum().backward()
    for a, b in zip(out[0], _grads(m)):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("L,H,B", [(2, 32, 32), (3, 16, 7)])
def test_lstm_fused_ce_matches_reference(L, H, B):
    """LSTM.loss on the GPU: the last step's mean CE fused into the forward kernel's tail (row
    loss, head gradient, ticketed fixed-order mean), the backward scaled by dloss — against the
    torch reference (reference_forward + F.cross_entropy); a scaled loss scales every gradient;
    the fused path is bit-reproducible."""
    torch.manual_seed(4)
    V, C, T, pad = 61, 4, 33, 3
    m = LSTM(V, H, H, C, num_layers=L, padding_idx=pad, dropout=0.3).cuda().train()
    ids = torch.randint(0, V, (B, T), device="cuda")
    y = torch.randint(0, C, (B,), device="cuda")
    params = m.param_list()
    seed = m.rng.current()
    loss, last = m.loss(ids, y)
    (2.5 * loss).backward()
    gk = _grads(m)
    for q in params:
        q.grad = None
    pr, _, _ = LS.reference_forward(ids, None, None, params, L, 0.3, seed, m.salt, pad)
    ref = torch.nn.functional.cross_entropy(pr[:, -1], y)
    (2.5 * ref).backward()
    assert abs(float(loss) - float(ref)) <= 1e-5 * abs(float(ref)) + 1e-6
    torch.testing.assert_close(last, pr[:, -1].detach(), rtol=1e-4, atol=1e-4)
    for a, b in zip(gk, _grads(m)):
        torch.testing.assert_close(a, b, rtol=2e-3, atol=2e-4)
    for q in params:
        q.grad = None
    loss2, _ = m.loss(ids, y)
    (2.5 * loss2).backward()
    assert float(loss2) == float(loss)
    for a, b in zip(gk, _grads(m)):
        assert torch.equal(a, b)
