"""Encoder-decoder Transformer translator (the reference's transformer.py), MI355X-native.

Module tree, attribute and parameter names match the reference exactly
(transformer.py:44-284), so a reference ``state_dict`` loads unchanged
(e.g. ``encoder.layers.0.attention.qkv_layer.weight``, ``decoder.layers.0.layer_norm1.gamma``,
``linear.weight``).  The per-head interleaved qkv / kv weight layouts (transformer.py:76-79,
:183-187) are kept, and the attention kernel reads them in place.

Each sublayer is one chain of fused ops (sparkmi.ops):
  linear(qkv) -> attention core -> linear(out) -> dropout+residual+LayerNorm
  linear1+ReLU+dropout -> linear2 -> dropout+residual+LayerNorm
GPU activation dtype per model: ``dtype="fp32"`` is the reference precision (fp32 activations and
weights, fp32-input MFMA GEMMs and attention); ``dtype="bf16"`` runs bf16 activations / bf16
weight shadow with fp32 master weights and fp32 accumulation.  CPU: fp32 torch math.

Mask semantics:
  mask_mode="reference" reproduces the reference numerically: the encoder padding mask is a
  no-op, the decoder self- and cross-attention "look-ahead" masks become a +1.0 bias on
  strictly-past keys.  mask_mode="causal" is the corrected semantics: key-padding masking in
  the encoder and cross attention, true causal masking in decoder self-attention.
"""
import functools
from dataclasses import dataclass


import torch
from torch import nn

from ..ops import (DropoutRNG, add_dropout_layernorm, cross_attention, embedding, linear, self_attention,
                   sinusoid_table)
from ..ops import _grad
from ..ops._grad import ResidualGrad
from ..ops._grad import SharedGrad
from ..ops.linear import concat_linear, ffn
from ..ops import planes as _pl
from ..ops.loss import cross_entropy
from ..ops.rng import new_salt, salt_scope


def get_device():
    """transformer.py:8-9."""
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


@dataclass
class TransformerConfig:
    d_model: int = 512
    ffn_hidden: int = 1024
    num_heads: int = 8
    drop_prob: float = 0.1
    num_layers: int = 1
    max_sequence_length: int = 200
    src_vocab_size: int = 10000
    tgt_vocab_size: int = 10000
    emb_dropout: float = 0.1          # SentenceEmbedding hard-codes p=0.1 (transformer.py:53)
    mask_mode: str = "reference"      # or "causal"
    pad_id: int = 0
    dtype: str = "bf16"               # GPU activation dtype: "bf16" (fp32 master) or "fp32" (reference precision)


def _native_path(x):
    from .. import _native
    return _native.use_native(x)


def _share(obj, name, value):
    object.__setattr__(obj, name, value)


class PositionalEncoding(nn.Module):
    """transformer.py:27-42; computed once and cached instead of on every forward (Q8)."""

    def __init__(self, d_model, max_sequence_length):
        super().__init__()
        self.max_sequence_length = max_sequence_length
        self.d_model = d_model
        self.register_buffer("table", sinusoid_table(max_sequence_length, d_model), persistent=False)

    def forward(self):
        return self.table


# The encoder's token embedding launches the queued grouped weight gradients at the start of its
# backward (sparkmi/ops/embedding.py), so the encoder's group runs beside the embedding sum.
ENC_EMB_FLUSH = True


class SentenceEmbedding(nn.Module):
    def __init__(self, max_sequence_length, d_model, vocab_size, rng, p=0.1, dtype="bf16"):
        super().__init__()
        self.act_dtype = dtype
        self.vocab_size = vocab_size
        self.max_sequence_length = max_sequence_length
        self.embedding = nn.Embedding(vocab_size, d_model)
        self.position_encoder = PositionalEncoding(d_model, max_sequence_length)
        self.dropout = nn.Dropout(p=p)
        _share(self, "_rng", rng)
        self.salt = new_salt()
        self.flush_wgrad = False  # the Encoder's: its backward ends the backward pass

    def forward(self, x):
        p = self.dropout.p if self.training else 0.0
        # the embedding's output dtype sets the dtype of every downstream fused op
        dtype = torch.bfloat16 if (x.is_cuda and self.act_dtype == "bf16") else torch.float32
        return embedding(x, self.embedding.weight, self.position_encoder.table, p, self._rng, self.salt,
                         out_dtype=dtype, flush_wgrad=self.flush_wgrad)



def transformer_flops_per_sample(layers, seq, vocab, d=512, ffn=1024):
    """Matmul FLOPs of one training sample (forward + backward = 3x forward): per token, each
    encoder layer's QKV / out-projection / FFN GEMMs, each decoder layer's self QKV / out, cross
    Q / KV / out and FFN GEMMs, the vocab projection, plus QK^T and PV of the 3 attention sites per
    layer pair (63.4 GFLOP at L6 S256 V10k).  The one definition bench.py and the
    translator recipe report TFLOP/s with."""
    enc = 2 * d * (3 * d + d + 2 * ffn)
    dec = 2 * d * (3 * d + d + d + 2 * d + d + 2 * ffn)
    attn = 3 * 4 * seq * d
    return 3 * (layers * (enc + dec + attn) + 2 * d * vocab) * seq


def _gp(t):
    """A sublayer-internal tensor with one consumer (attention core / LayerNorm / loss): its
    gradient may come back as split planes only (sparkmi/ops/planes.py, SMI_PLANES_ONLY)."""
    return _pl.mark_grad_planes_ok(t)


class MultiHeadAttention(nn.Module):
    def __init__(self, d_model, num_heads):
        super().__init__()
        self.d_model = d_model
        self.num_heads = num_heads
        self.head_dim = d_model // num_heads
        self.qkv_layer = nn.Linear(d_model, 3 * d_model)
        self.linear_layer = nn.Linear(d_model, d_model)

    def forward(self, x, mode="none", key_padding=None, x_slot=None):
        qkv = _gp(linear(x, self.qkv_layer.weight, self.qkv_layer.bias, x_slot=x_slot))
        values = self_attention(qkv, self.num_heads, mode, key_padding)
        return _gp(linear(values, self.linear_layer.weight, self.linear_layer.bias))


class MultiHeadCrossAttention(nn.Module):
    def __init__(self, d_model, num_heads):
        super().__init__()
        self.d_model = d_model
        self.num_heads = num_heads
        self.head_dim = d_model // num_heads
        self.kv_layer = nn.Linear(d_model, 2 * d_model)
        self.q_layer = nn.Linear(d_model, d_model)
        self.linear_layer = nn.Linear(d_model, d_model)

    def forward(self, x, y, mode="none", key_padding=None, y_slot=None, kv=None):
        """``kv``: optional (kv_all, column, SharedGrad) — this layer's k/v projection already
        computed inside the decoder's concatenated kv GEMM (Decoder._shared_kv)."""
        if kv is None:
            kv_all = _gp(linear(x, self.kv_layer.weight, self.kv_layer.bias))
            col, shared = 0, None
        else:
            kv_all, col, shared = kv
        q = _gp(linear(y, self.q_layer.weight, self.q_layer.bias, x_slot=y_slot))
        values = cross_attention(q, kv_all, self.num_heads, mode, key_padding, col, shared)
        return _gp(linear(values, self.linear_layer.weight, self.linear_layer.bias))


class LayerNormalization(nn.Module):
    """transformer.py:86-101 (parameter names gamma/beta kept)."""

    def __init__(self, parameters_shape, eps=1e-5):
        super().__init__()
        self.parameters_shape = list(parameters_shape)
        self.eps = eps
        self.gamma = nn.Parameter(torch.ones(parameters_shape))
        self.beta = nn.Parameter(torch.zeros(parameters_shape))

    def forward(self, inputs, residual=None, p=0.0, rng=None, salt=0, r_slot=None):
        return add_dropout_layernorm(inputs, residual, self.gamma, self.beta, p, rng, salt, self.eps, r_slot)


class PositionwiseFeedForward(nn.Module):
    def __init__(self, d_model, hidden, drop_prob=0.1, rng=None):
        super().__init__()
        self.linear1 = nn.Linear(d_model, hidden)
        self.linear2 = nn.Linear(hidden, d_model)
        self.relu = nn.ReLU()
        self.dropout = nn.Dropout(p=drop_prob)
        _share(self, "_rng", rng)
        self.salt = new_salt()

    def forward(self, x, x_slot=None):
        p = self.dropout.p if self.training else 0.0
        return _gp(ffn(x, self.linear1, self.linear2, p, self._rng, self.salt, x_slot))


class EncoderLayer(nn.Module):
    def __init__(self, d_model, ffn_hidden, num_heads, drop_prob, rng):
        super().__init__()
        self.attention = MultiHeadAttention(d_model=d_model, num_heads=num_heads)
        self.norm1 = LayerNormalization(parameters_shape=[d_model])
        self.dropout1 = nn.Dropout(p=drop_prob)
        self.ffn = PositionwiseFeedForward(d_model=d_model, hidden=ffn_hidden, drop_prob=drop_prob, rng=rng)
        self.norm2 = LayerNormalization(parameters_shape=[d_model])
        self.dropout2 = nn.Dropout(p=drop_prob)
        _share(self, "_rng", rng)
        self.salts = (new_salt(), new_salt())

    def forward(self, x, mode="none", key_padding=None):
        p1 = self.dropout1.p if self.training else 0.0
        p2 = self.dropout2.p if self.training else 0.0
        # residual gradients ride the dgrad epilogue of the block's first linear (ResidualGrad)
        s1, s2 = ResidualGrad(), ResidualGrad()
        a = self.attention(x, mode, key_padding, x_slot=s1)
        x = self.norm1(a, x, p1, self._rng, self.salts[0], r_slot=s1)
        f = self.ffn(x, x_slot=s2)
        return self.norm2(f, x, p2, self._rng, self.salts[1], r_slot=s2)


def _mid_flush(g):
    _grad.flush_groups_async(g.device)


def _flush_depths(k):
    """A *_MID_FLUSH setting as a set of depths: an int k (0: none) or a string "k1-k2-..." (a
    flush after each of those many top layers)."""
    if isinstance(k, str):
        return {int(v) for v in k.split("-") if v}
    return {int(k)} if k else set()


# The top ENC_MID_FLUSH encoder layers' queued weight gradients go to the side stream once their
# backward is done (0: with the rest, launched by the encoder embedding's backward).  In-step A/B
# (profiles/r6_dec_mid_flush_ab.txt): bf16 4 layers -0.15 ms (the lower layers' backward runs
# beside them and the final group is shorter); fp32 +0.06..0.3 ms (its long compute-bound group
# tiles starve the lower layers' dgrad chain), so fp32 keeps one group
ENC_MID_FLUSH = 0
ENC_MID_FLUSH_BF16 = 4


class SequentialEncoder(nn.Sequential):
    def forward(self, *inputs):
        x, mode, key_padding = inputs
        n = len(self._modules)
        ks = _flush_depths(ENC_MID_FLUSH_BF16 if x.dtype == torch.bfloat16 else ENC_MID_FLUSH)
        for i, module in enumerate(self._modules.values()):
            if n - i in ks and x.requires_grad and torch.is_grad_enabled():
                x.register_hook(_mid_flush)
            x = module(x, mode, key_padding)
        return x


class Encoder(nn.Module):
    def __init__(self, d_model, ffn_hidden, num_heads, drop_prob, num_layers, max_sequence_length, vocab_size, rng,
                 emb_dropout=0.1, dtype="bf16"):
        super().__init__()
        self.sentence_embedding = SentenceEmbedding(max_sequence_length, d_model, vocab_size, rng, emb_dropout, dtype)
        self.sentence_embedding.flush_wgrad = ENC_EMB_FLUSH
        self.layers = SequentialEncoder(*[EncoderLayer(d_model, ffn_hidden, num_heads, drop_prob, rng)
                                          for _ in range(num_layers)])

    def forward(self, x, mode="none", key_padding=None):
        x = self.sentence_embedding(x)
        return self.layers(x, mode, key_padding)


class DecoderLayer(nn.Module):
    def __init__(self, d_model, ffn_hidden, num_heads, drop_prob, rng):
        super().__init__()
        self.self_attention = MultiHeadAttention(d_model=d_model, num_heads=num_heads)
        self.layer_norm1 = LayerNormalization(parameters_shape=[d_model])
        self.dropout1 = nn.Dropout(p=drop_prob)
        self.encoder_decoder_attention = MultiHeadCrossAttention(d_model=d_model, num_heads=num_heads)
        self.layer_norm2 = LayerNormalization(parameters_shape=[d_model])
        self.dropout2 = nn.Dropout(p=drop_prob)
        self.ffn = PositionwiseFeedForward(d_model=d_model, hidden=ffn_hidden, drop_prob=drop_prob, rng=rng)
        self.layer_norm3 = LayerNormalization(parameters_shape=[d_model])
        self.dropout3 = nn.Dropout(p=drop_prob)
        _share(self, "_rng", rng)
        self.salts = (new_salt(), new_salt(), new_salt())

    def forward(self, x, y, self_mode="none", cross_mode="none", key_padding=None, kv=None):
        ps = [d.p if self.training else 0.0 for d in (self.dropout1, self.dropout2, self.dropout3)]
        s1, s2, s3 = ResidualGrad(), ResidualGrad(), ResidualGrad()
        a = self.self_attention(y, self_mode, x_slot=s1)
        y = self.layer_norm1(a, y, ps[0], self._rng, self.salts[0], r_slot=s1)
        c = self.encoder_decoder_attention(x, y, cross_mode, key_padding, y_slot=s2, kv=kv)
        y = self.layer_norm2(c, y, ps[1], self._rng, self.salts[1], r_slot=s2)
        f = self.ffn(y, x_slot=s3)
        return self.layer_norm3(f, y, ps[2], self._rng, self.salts[2], r_slot=s3)


# The top DEC_MID_FLUSH decoder layers' queued weight gradients (and the vocabulary projection's)
# go to the side stream as soon as those layers' backward is done, instead of with the rest at the
# decoder/encoder cut (0: one group at the cut).  In-step A/B (profiles/r6_dec_mid_flush_ab.txt):
# fp32 4 layers -0.06 ms (the first group overlaps the lower decoder layers' backward, the group
# at the cut is smaller); bf16 +0.04 ms at 4, so bf16 (DEC_MID_FLUSH_BF16) keeps one group
DEC_MID_FLUSH = 4
DEC_MID_FLUSH_BF16 = 0


class SequentialDecoder(nn.Sequential):
    def forward(self, *inputs):
        x, y, self_mode, cross_mode, key_padding = inputs[:5]
        kvs = inputs[5] if len(inputs) > 5 and inputs[5] is not None else [None] * len(self._modules)
        n = len(self._modules)
        ks = _flush_depths(DEC_MID_FLUSH_BF16 if y.dtype == torch.bfloat16 else DEC_MID_FLUSH)
        for i, (module, kv) in enumerate(zip(self._modules.values(), kvs)):
            if n - i in ks and y.requires_grad and torch.is_grad_enabled():
                y.register_hook(_mid_flush)
            y = module(x, y, self_mode, cross_mode, key_padding, kv)
        return y


class Decoder(nn.Module):
    def __init__(self, d_model, ffn_hidden, num_heads, drop_prob, num_layers, max_sequence_length, vocab_size, rng,
                 emb_dropout=0.1, dtype="bf16"):
        super().__init__()
        self.sentence_embedding = SentenceEmbedding(max_sequence_length, d_model, vocab_size, rng, emb_dropout, dtype)
        self.layers = SequentialDecoder(*[DecoderLayer(d_model, ffn_hidden, num_heads, drop_prob, rng)
                                          for _ in range(num_layers)])

    def forward(self, x, y, self_mode="none", cross_mode="none", key_padding=None, flat=None):
        y = self.sentence_embedding(y)
        return self.layers(x, y, self_mode, cross_mode, key_padding, self._shared_kv(x, flat))

    def kv_linears(self):
        return [l.encoder_decoder_attention.kv_layer for l in self.layers]

    def _shared_kv(self, x, flat):
        """Every decoder layer projects the SAME encoder output to k/v (transformer.py:175-182):
        on the GPU, with the kv weights stored back to back (Transformer._smi_flat_groups), that is
        ONE GEMM of width L*2D; each layer's cross attention reads its column block and writes its
        k/v gradient into the shared buffer, so the backward is one dgrad GEMM (K = L*2D, the sum
        over layers done in the accumulators) and one weight-gradient GEMM."""
        lins = self.kv_linears()
        if flat is None or len(lins) < 2 or not _native_path(x):
            return None
        shared = SharedGrad()
        kv_all = concat_linear(x, flat, lins, shared)
        if kv_all is None:
            return None
        cols = [0]
        for l in lins[:-1]:
            cols.append(cols[-1] + l.weight.shape[0])
        return [(kv_all, c, shared) for c in cols]


class Transformer(nn.Module):
    """transformer.py:255-284.  ``forward(x, y, ...)`` returns logits [B, S, tgt_vocab]."""

    def __init__(self, d_model=512, ffn_hidden=1024, num_heads=8, drop_prob=0.1, num_layers=1,
                 max_sequence_length=200, de_vocab_size=10000, src_vocab_size=None, tgt_vocab_size=None,
                 mask_mode="reference", emb_dropout=0.1, pad_id=0, seed=0, dtype="bf16", salt_base=1):
        super().__init__()
        if dtype not in ("bf16", "fp32"):
            raise ValueError(f"dtype must be 'bf16' or 'fp32', got {dtype!r}")
        src_vocab_size = src_vocab_size or de_vocab_size
        tgt_vocab_size = tgt_vocab_size or de_vocab_size
        self.config = TransformerConfig(d_model, ffn_hidden, num_heads, drop_prob, num_layers, max_sequence_length,
                                        src_vocab_size, tgt_vocab_size, emb_dropout, mask_mode, pad_id, dtype)
        self.rng = DropoutRNG(seed)
        with salt_scope(salt_base):  # the model's own dropout-salt stream (sparkmi/ops/rng.py)
            self.encoder = Encoder(d_model, ffn_hidden, num_heads, drop_prob, num_layers, max_sequence_length,
                                   src_vocab_size, self.rng, emb_dropout, dtype)
            self.decoder = Decoder(d_model, ffn_hidden, num_heads, drop_prob, num_layers, max_sequence_length,
                                   tgt_vocab_size, self.rng, emb_dropout, dtype)
        self.linear = nn.Linear(d_model, tgt_vocab_size)

    def _smi_flat_groups(self):
        """FlatParams layout hint: the decoder's kv projections back to back (Decoder._shared_kv)."""
        lins = self.decoder.kv_linears()
        return [[l.weight for l in lins], [l.bias for l in lins]]

    @classmethod
    def from_config(cls, cfg: TransformerConfig, seed=0):
        return cls(cfg.d_model, cfg.ffn_hidden, cfg.num_heads, cfg.drop_prob, cfg.num_layers,
                   cfg.max_sequence_length, cfg.tgt_vocab_size, cfg.src_vocab_size, cfg.tgt_vocab_size,
                   cfg.mask_mode, cfg.emb_dropout, cfg.pad_id, seed, cfg.dtype)

    def _modes(self, x, encoder_self_attention_mask, decoder_self_attention_mask, decoder_cross_attention_mask,
               y=None):
        if self.config.mask_mode == "reference":
            # the masks are read by value, as the reference adds them (transformer.py:17-19)
            Ss = x.shape[1]
            St = y.shape[1] if y is not None else Ss
            enc_mode, kp = interpret_mask(encoder_self_attention_mask, Ss, Ss)
            self_mode, kp_self = interpret_mask(decoder_self_attention_mask, St, St)
            cross_mode, kp_cross = interpret_mask(decoder_cross_attention_mask, St, Ss)
            if kp_self is not None:
                raise ValueError("decoder self-attention: key-padding masks are not supported by the fused kernels")
            if kp is not None and kp_cross is not None and not torch.equal(kp, kp_cross):
                raise ValueError("encoder and cross-attention key-padding masks must agree")
            kp = kp if kp is not None else kp_cross
            if kp is not None:
                kp = kp.to(x.device)
            return enc_mode, self_mode, cross_mode, kp
        key_padding = (x == self.config.pad_id)
        return "none", "causal", "none", key_padding

    def forward(self, x, y, encoder_self_attention_mask=None, decoder_self_attention_mask=None,
                decoder_cross_attention_mask=None, enc_key_padding=None):
        enc_mode, self_mode, cross_mode, kp = self._modes(x, encoder_self_attention_mask,
                                                          decoder_self_attention_mask, decoder_cross_attention_mask, y)
        if enc_key_padding is not None:
            kp = enc_key_padding
        x = self.encoder(x, enc_mode, kp)
        out = self.decoder(x, y, self_mode, cross_mode, kp, getattr(self, "_smi_flat", None))
        # fp32 GPU: the epilogue also reduces each logits row (softmax statistics per 128 columns),
        # so the cross-entropy forward never re-reads the logits (sparkmi/ops/loss.py)
        return linear(out, self.linear.weight, self.linear.bias)

    def loss(self, logits, target):
        """Token CE ignoring pad, mean over non-pad targets (pytorch_machine_translator.py:182-188)."""
        return cross_entropy(logits, target, ignore_index=self.config.pad_id)

    def training_step_loss(self, src, tgt, shift_targets=False):
        """Reference recipe (Q7: decoder input == target, no shift) or shifted teacher forcing."""
        if shift_targets:
            dec_in, target = tgt[:, :-1], tgt[:, 1:]
        else:
            dec_in, target = tgt, tgt
        la = create_look_ahead_mask(dec_in.shape[1])  # the reference's decoder masks (host, cached)
        logits = _gp(self(src, dec_in, None, la, la))  # consumed by the loss only
        return self.loss(logits, target)

    def training_step_split(self, src, tgt, shift_targets=False, enc_cuts=None):
        """The same loss with the autograd graph cut into segments, for a backward in several
        pieces (``StepRunner(split_fn=...)``): the encoder output and the encoder layer outputs
        listed in ``enc_cuts`` (default: the middle layer) become detached leaves.  Returns
        ``(loss, segments)`` with ``segments = [(leaf, root), ...]`` in BACKWARD order:
        ``loss.backward()`` finishes every decoder / vocab-projection gradient and leaves the
        top leaf's gradient; then, for each segment, ``root.backward(leaf.grad)`` runs the next
        slice of the encoder backward.  A data-parallel step all-reduces the gradient buckets
        that are final after each piece while the next piece runs."""
        if shift_targets:
            dec_in, target = tgt[:, :-1], tgt[:, 1:]
        else:
            dec_in, target = tgt, tgt
        la = create_look_ahead_mask(dec_in.shape[1])
        enc_mode, self_mode, cross_mode, kp = self._modes(src, None, la, la, dec_in)
        layers = list(self.encoder.layers)
        n = len(layers)
        cuts = sorted({c for c in (enc_cuts if enc_cuts is not None else [n // 2]) if 0 < c < n})
        x = self.encoder.sentence_embedding(src)
        segments, start = [], 0
        for c in cuts + [n]:
            for layer in layers[start:c]:
                x = layer(x, enc_mode, kp)
            leaf = x.detach().requires_grad_()
            segments.append((leaf, x))
            x, start = leaf, c
        out = self.decoder(x, dec_in, self_mode, cross_mode, kp, getattr(self, "_smi_flat", None))
        logits = _gp(linear(out, self.linear.weight, self.linear.bias))
        return self.loss(logits, target), segments[::-1]


@functools.lru_cache(maxsize=16)
def create_look_ahead_mask(size):
    """pytorch_machine_translator.py:102-104 (bool [1,1,S,S], True above the diagonal); cached
    host tensor, so the per-step mask costs nothing and is interpreted once."""
    mask = torch.tril(torch.ones(size, size)) == 0
    return mask.unsqueeze(0).unsqueeze(0)


_NEG = -1e4  # an additive bias at or below this is a "masked out" key
_mask_cache = {}


def interpret_mask(mask, Sq, Sk):
    """What the fused attention kernels must do for a reference-style mask tensor.

    The reference ADDS ``mask.permute(0, 1, 3, 2)`` to the [B, H, Sq, Sk] scores
    (transformer.py:17-19); bool masks add 1.0 where True.  Returns ``(mode, key_padding)``:
      * None, or a bias constant along each score row (e.g. the [B,1,1,S] padding mask, which
        becomes [B,1,S,1]): softmax is shift-invariant -> "none";
      * +1.0 exactly on strictly-past keys (the look-ahead mask of
        pytorch_machine_translator.py:102-104 after the permute) -> "reference";
      * large negative (<= -1e4 or -inf) on future keys and row-constant elsewhere -> "causal";
      * large negative on a per-(batch, key) set, row-constant elsewhere -> key padding [B, Sk]
        (optionally with the causal pattern);
    anything else raises ValueError: there is no general additive-bias attention kernel.
    Device masks are read once per distinct tensor version (cached)."""
    if mask is None:
        return "none", None
    if not torch.is_tensor(mask) or mask.dim() != 4:
        raise ValueError("attention masks must be 4-D tensors added to the scores after permute(0, 1, 3, 2) "
                         f"(transformer.py:17-19); got {type(mask).__name__} "
                         f"{tuple(mask.shape) if torch.is_tensor(mask) else ''}")
    B, H, Kd, Qd = mask.shape  # after the permute: [B, H, Qd, Kd]
    if Qd not in (1, Sq) or Kd not in (1, Sk):
        raise ValueError(f"mask of shape {tuple(mask.shape)} does not broadcast over scores [.., {Sq}, {Sk}]")
    if Kd == 1:  # constant along every score row: a softmax no-op, decided from the shape alone
        return "none", None
    key = (mask.data_ptr(), mask._version, tuple(mask.shape), mask.dtype, str(mask.device), Sq, Sk)
    hit = _mask_cache.get(key)
    if hit is not None:
        return hit
    b = mask.detach().to("cpu", torch.float64).permute(0, 1, 3, 2)
    if H > 1 and not torch.equal(b, b[:, :1].expand_as(b)):
        raise ValueError("per-head attention masks are not supported by the fused kernels")
    b = b[:, 0].expand(B, Sq, Sk)
    q = torch.arange(Sq).view(Sq, 1)
    k = torch.arange(Sk).view(1, Sk)
    past = (k < q).to(torch.float64)
    neg = b <= _NEG

    def row_const(t, where):
        t = torch.where(where, t, t.new_full((), float("nan")))
        hi = torch.nan_to_num(t, nan=-float("inf")).amax(-1)
        lo = torch.nan_to_num(t, nan=float("inf")).amin(-1)
        return bool(((hi == lo) | torch.isinf(hi)).all())

    out = None
    every = torch.ones_like(neg)
    if not neg.any():
        if row_const(b, every):
            out = ("none", None)
        elif row_const(b - past, every):
            out = ("reference", None)
    elif row_const(b, ~neg):
        future = (k > q).expand(B, Sq, Sk)
        kp = neg.all(1)  # keys masked for every query row: key padding [B, Sk]
        rest = neg & ~kp[:, None, :]
        kpo = kp if bool(kp.any()) else None
        if not rest.any():
            out = ("none", kpo)
        elif torch.equal(rest, future & ~kp[:, None, :]):
            out = ("causal", kpo)
    if out is None:
        raise ValueError("unsupported attention mask: the fused kernels implement no-op (row-constant), the "
                         "reference look-ahead (+1 on past keys), causal and key-padding masks")
    if len(_mask_cache) > 64:
        _mask_cache.clear()
    _mask_cache[key] = out
    return out
