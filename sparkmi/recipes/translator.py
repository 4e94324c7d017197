"""English -> German Transformer training — pytorch_machine_translator.py (R39-R41) with the
model of transformer.py (R24-R38), single executor or data-parallel over N MI355X executors
(the latter is new capability, BASELINE.json).

Reference: d_model 512, ffn 1024, 8 heads, dropout 0.1, 1 layer, S = 200 (Truncate(199) +
<sos>/<eos> + PadTransform(200)), batch 32, 1 epoch, Adam 1e-3, token CE ignoring <pad> with a
masked mean, decoder input == target (no shift, Q7), the reference's mask semantics (Q6:
padding mask no-op, look-ahead mask adds +1.0 to strictly-past keys).  ``--shift-targets`` and
``--mask-mode causal`` select the textbook variants instead.  spaCy tokenizers are unavailable
offline, so both sides use basic_english (X14).  ``--dtype fp32`` (default) trains at the
reference's precision (fp32 modules, pytorch_machine_translator.py:120-137); ``--dtype bf16``
runs bf16 activations with fp32 master weights.  Data-parallel runs capture the backward as
several graphs so finished gradient buckets are reduced under the rest of the backward.
"""
import dataclasses

import torch

from ..data.dataset import DeviceLoader
from ..data.synthetic import translation_text
from ..data.text import build_vocab_from_iterator, get_tokenizer, text_pipeline
from ..models.transformer import Transformer, transformer_flops_per_sample
from ..optim import Adam
from ..train.config import TrainConfig, parse
from ..train.trainer import Trainer, setup_executor
from .common import run, shard

SPECIALS = ["<pad>", "<sos>", "<eos>", "<unk>"]


@dataclasses.dataclass
class TranslatorConfig(TrainConfig):
    """Transformer translator (pytorch_machine_translator.py)."""
    epochs: int = 1
    batch_size: int = 32
    lr: float = 1e-3
    d_model: int = 512
    ffn_hidden: int = 1024
    num_heads: int = 8
    drop_prob: float = 0.1
    num_layers: int = 1
    max_sequence_length: int = 200
    mask_mode: str = "reference"
    dtype: str = "fp32"            # "fp32" (reference precision) | "bf16" (bf16 activations, fp32 master)
    shift_targets: bool = False
    n_train: int = 29000
    log_every: int = 100


def build_corpus(cfg):
    pairs = translation_text(cfg.n_train, seed=cfg.seed)
    tok = get_tokenizer("basic_english")
    en_tok = [tok(e) for e, _ in pairs]
    de_tok = [tok(d) for _, d in pairs]
    en_vocab = build_vocab_from_iterator(iter(en_tok), min_freq=1, specials=SPECIALS, special_first=True)
    de_vocab = build_vocab_from_iterator(iter(de_tok), min_freq=1, specials=SPECIALS, special_first=True)
    en_vocab.set_default_index(en_vocab["<unk>"])
    de_vocab.set_default_index(en_vocab["<unk>"])  # as the reference (:67)
    S = cfg.max_sequence_length
    en_pipe = text_pipeline(en_vocab, 1, 2, S - 1, 0, pad_to=S)
    de_pipe = text_pipeline(de_vocab, 1, 2, S - 1, 0, pad_to=S)
    return en_vocab, de_vocab, en_pipe(en_tok)[:, :S].contiguous(), de_pipe(de_tok)[:, :S].contiguous()


def train_fn(cfg):
    rank, world, device = setup_executor(cfg)
    en_vocab, de_vocab, src, tgt = build_corpus(cfg)
    idx = torch.from_numpy(shard(len(src), rank, world, cfg.seed))
    loader = DeviceLoader([src[idx], tgt[idx]], cfg.batch_size, device, shuffle=True, drop_last=True,
                          seed=cfg.seed + 1000 * rank)
    torch.manual_seed(cfg.seed)
    if cfg.dtype not in ("fp32", "bf16"):
        raise ValueError(f"--dtype must be fp32 or bf16, got {cfg.dtype!r}")
    model = Transformer(cfg.d_model, cfg.ffn_hidden, cfg.num_heads, cfg.drop_prob, cfg.num_layers,
                        cfg.max_sequence_length, len(de_vocab), len(en_vocab), len(de_vocab), mask_mode=cfg.mask_mode,
                        seed=cfg.seed + rank, dtype=cfg.dtype)
    shift = cfg.shift_targets
    S = cfg.max_sequence_length - (1 if shift else 0)
    flops = transformer_flops_per_sample(cfg.num_layers, S, len(de_vocab), cfg.d_model, cfg.ffn_hidden)
    trainer = Trainer(model, lambda m, s, t: m.training_step_loss(s, t, shift_targets=shift),
                      lambda flat: Adam(flat, lr=cfg.lr), cfg, device, rank, world, "translator",
                      shadow=(cfg.dtype == "bf16" and torch.device(device).type == "cuda"),
                      split_fn=lambda m, s, t: m.training_step_split(s, t, shift_targets=shift),
                      flops_per_sample=flops)
    stats = trainer.fit(loader, cfg.epochs)
    trainer.close()
    out = dict(stats, world=world, en_vocab=len(en_vocab), de_vocab=len(de_vocab), dtype=cfg.dtype)
    if rank == 0:
        out["train_samples_per_s"] = stats["steps"] * cfg.batch_size * world / max(stats["time_s"], 1e-9)
    return out if rank == 0 else None


def main(argv=None):
    cfg = parse(TranslatorConfig, argv)
    res = run(train_fn, cfg)
    if cfg.verbose and res is not None:
        print(res)
    return res


if __name__ == "__main__":
    main()
