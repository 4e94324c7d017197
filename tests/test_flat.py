"""FlatParams layout (sparkmi/utils/flat.py) on CPU: reverse registration order, 64-element
alignment, and parameter groups stored back to back (the decoder kv projections that the GPU
path runs as one GEMM, sparkmi/models/transformer.py Decoder._shared_kv)."""
import torch

from sparkmi.utils.flat import ALIGN, FlatParams


def _model(L=3):
    from sparkmi.models.transformer import Transformer
    torch.manual_seed(0)
    return Transformer(d_model=64, ffn_hidden=128, num_heads=1, num_layers=L, max_sequence_length=16,
                       src_vocab_size=40, tgt_vocab_size=40)


def test_kv_group_back_to_back_and_views():
    m = _model()
    ref = {n: p.detach().clone() for n, p in m.named_parameters()}
    flat = FlatParams(m)
    lins = m.decoder.kv_linears()
    wv = flat.concat([l.weight for l in lins])
    bv = flat.concat([l.bias for l in lins])
    assert wv is not None and bv is not None
    W = wv[0].view(-1, 64)
    assert torch.equal(W, torch.cat([l.weight.detach() for l in lins]))
    assert torch.equal(bv[0], torch.cat([l.bias.detach() for l in lins]))
    # gradient views alias the parameters' .grad
    wv[1].view(-1, 64)[: lins[0].weight.shape[0]].fill_(1.0)
    assert torch.all(lins[0].weight.grad == 1.0) and torch.all(lins[1].weight.grad == 0.0)
    # values preserved, every parameter aligned, reversed order outside the group
    for n, p in m.named_parameters():
        assert torch.equal(p.detach(), ref[n]), n
        assert flat.param_range(p)[0] % ALIGN == 0
    assert flat.names[0] == "linear.bias"
    # the group sits where its first-registered member (decoder layer 0) would
    i0 = flat.names.index("decoder.layers.0.encoder_decoder_attention.kv_layer.weight")
    assert flat.names[i0 + 1] == "decoder.layers.1.encoder_decoder_attention.kv_layer.weight"
    assert (flat.names.index("decoder.layers.0.encoder_decoder_attention.q_layer.weight") < i0
            < flat.names.index("decoder.layers.0.layer_norm1.gamma"))


def test_concat_rejects_non_contiguous():
    m = _model()
    flat = FlatParams(m)
    lins = m.decoder.kv_linears()
    assert flat.concat([lins[1].weight, lins[0].weight]) is None
    assert flat.concat([lins[0].weight, lins[0].bias]) is None


def test_groups_skipped_when_padding_breaks_contiguity():
    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Parameter(torch.zeros(10))  # not a multiple of ALIGN
            self.b = torch.nn.Parameter(torch.zeros(64))

        def _smi_flat_groups(self):
            return [[self.a, self.b]]
    flat = FlatParams(M())
    assert flat.names == ["b", "a"]


def test_cpu_training_unchanged_by_grouping():
    """The CPU path never takes the fused kv GEMM; with or without flat storage the loss and
    gradients are identical."""
    from sparkmi.data.synthetic import translation_pairs
    src, tgt = translation_pairs(2, 16, 40, 40, seed=1)
    import copy
    a = _model()
    b = copy.deepcopy(a)  # same dropout salts
    FlatParams(b)
    la, lb = a.training_step_loss(src, tgt), b.training_step_loss(src, tgt)
    la.backward()
    lb.backward()
    assert torch.equal(la, lb)
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        torch.testing.assert_close(pa.grad, pb.grad, rtol=0, atol=0, msg=n)


def test_load_state_dict_refreshes_shadow_and_planes():
    """a direct module.load_state_dict (not through the checkpoint manager) re-derives
    the bf16 shadow and the fp32 GEMMs' weight planes from the new master weights."""
    import torch
    from sparkmi.utils.flat import FlatParams
    torch.manual_seed(0)
    m = torch.nn.Linear(16, 8)
    flat = FlatParams(m, device="cpu", shadow=True)
    flat.ensure_planes()
    sd = {k: torch.randn_like(v) for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    assert torch.equal(m.weight.detach(), sd["weight"])
    assert torch.equal(flat.shadow, flat.master.to(torch.bfloat16))
    p = flat.planes
    assert torch.equal(p[0].float() + p[1].float() + p[2].float(), flat.master)
