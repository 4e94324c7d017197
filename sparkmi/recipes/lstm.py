"""AG_NEWS LSTM text classification — distributed_lstm.py (R16-R22) and pytorch_lstm.py (R23).

Reference: basic_english tokenizer, vocab with specials <pad>,<sos>,<eos>,<unk> first, transform
Vocab -> <sos> -> Truncate(128) -> <eos> -> ToTensor(pad 0) (batches padded to their longest
sequence), LSTM(vocab, 32, 32, 4, num_layers=2, dropout 0.5), Adam lr 1e-3, CE on pred[:, -1],
3 epochs, batch 32, labels - 1 (distributed_lstm.py:56-205).

Here the corpus is tokenised + encoded ONCE by the C++ text pipeline into an HBM-resident padded
id matrix; each batch is a device gather trimmed to the batch's longest sequence (the same
shapes as the reference's per-batch ToTensor), and a step is the persistent fused LSTM
forward + BPTT kernels, CE on the last step and the fused Adam update.  The embedding's
padding_idx is ``vocab['0']`` like the reference (Q10).
"""
import dataclasses
import math

import numpy as np
import torch

from ..data.dataset import gather_rows
from ..data.synthetic import ag_news_text
from ..data.text import build_vocab_from_iterator, get_tokenizer, text_pipeline
from ..models.lstm import LSTM
from ..optim import Adam
from ..train.config import TrainConfig, parse
from ..train.trainer import Trainer, setup_executor
from .common import run, shard

SPECIALS = ["<pad>", "<sos>", "<eos>", "<unk>"]


@dataclasses.dataclass
class LSTMConfig(TrainConfig):
    """AG_NEWS LSTM classifier (distributed_lstm.py / pytorch_lstm.py)."""
    local_mode: bool = False       # TorchDistributor(local_mode=False), distributed_lstm.py:211-214
    epochs: int = 3
    batch_size: int = 32
    lr: float = 1e-3
    max_len: int = 128
    hidden_size: int = 32
    num_layers: int = 2
    output_dim: int = 4
    n_train: int = 120000
    n_test: int = 7600
    graph: bool = False          # batch length varies (padded to the longest in the batch)


class TextBatches:
    """Epoch-seeded batches of (ids[:, :T_batch], labels) from an HBM-resident padded id matrix;
    T_batch comes from host-side lengths, so no device sync per batch."""

    def __init__(self, ids, lengths, labels, batch_size, device, seed=0, shuffle=True):
        self.ids = ids.to(device)
        self.labels = labels.to(device)
        self.lengths = np.asarray(lengths)
        self.batch_size, self.seed, self.shuffle = batch_size, seed, shuffle
        self.device = device
        self.epoch, self.skip = 0, 0

    def set_epoch(self, e):
        self.epoch = e

    def __len__(self):
        return len(self.lengths) // self.batch_size  # drop_last=True (distributed_lstm.py:153)

    def __iter__(self):
        n = len(self.lengths)
        order = np.random.default_rng(self.seed + self.epoch).permutation(n) if self.shuffle else np.arange(n)
        start, self.skip = self.skip, 0
        for b in range(start, len(self)):
            sel = order[b * self.batch_size:(b + 1) * self.batch_size]
            T = int(self.lengths[sel].max())
            idx = torch.from_numpy(sel).to(self.device, non_blocking=True)
            x = gather_rows(self.ids, idx)[:, :T].contiguous()
            yield x, gather_rows(self.labels, idx)


def build_corpus(cfg):
    train = ag_news_text(cfg.n_train, seed=cfg.seed)
    test = ag_news_text(cfg.n_test, seed=cfg.seed + 1)
    tok = get_tokenizer("basic_english")
    vocab = build_vocab_from_iterator((tok(t) for _, t in train), min_freq=1, specials=SPECIALS, special_first=True)
    vocab.set_default_index(vocab["<unk>"])
    pipe = text_pipeline(vocab, sos=1, eos=2, max_len=cfg.max_len, pad=0)

    def encode(pairs):
        ids = pipe([tok(t) for _, t in pairs])
        lengths = (ids != 0).sum(1).numpy()
        labels = torch.tensor([lab - 1 for lab, _ in pairs], dtype=torch.int64)  # labels - 1 (:180)
        return ids, lengths, labels

    return vocab, encode(train), encode(test)


def train_fn(cfg):
    rank, world, device = setup_executor(cfg)
    vocab, (ids, lens, labels), (tids, tlens, tlabels) = build_corpus(cfg)
    sel = shard(len(labels), rank, world, cfg.seed)
    sel_t = torch.from_numpy(sel)
    loader = TextBatches(ids[sel_t], lens[sel], labels[sel_t], cfg.batch_size, device, seed=cfg.seed + 1000 * rank)
    torch.manual_seed(cfg.seed)
    pad = vocab["0"]  # the reference's padding_idx (distributed_lstm.py:115)
    model = LSTM(len(vocab), cfg.hidden_size, cfg.hidden_size, cfg.output_dim, cfg.num_layers, padding_idx=pad,
                 seed=cfg.seed)

    def loss_fn(m, x, y):
        loss, _ = m.loss(x, y)
        return loss

    # sparse exchange list capacity: <sos> + at most max_len tokens + <eos> per sequence
    trainer = Trainer(model, loss_fn, lambda flat: Adam(flat, lr=cfg.lr), cfg, device, rank, world, "lstm",
                      shadow=False, sparse_cap=cfg.batch_size * (cfg.max_len + 2))
    stats = trainer.fit(loader, cfg.epochs)
    trainer.close()
    out = dict(stats, world=world, vocab_size=len(vocab), padding_idx=pad)
    if rank == 0:
        model.eval()
        correct, n = 0, 0
        with torch.no_grad():
            test = TextBatches(tids, tlens, tlabels, 256, device, shuffle=False)
            for x, y in test:
                pred, _, _ = model(x)
                correct += (pred[:, -1].argmax(1) == y).sum().item()
                n += len(y)
        out["test_acc"] = 100.0 * correct / max(1, n)
        out["train_samples_per_s"] = stats["steps"] * cfg.batch_size * world / max(stats["time_s"], 1e-9)
    return out if rank == 0 else None


def main(argv=None):
    cfg = parse(LSTMConfig, argv)
    res = run(train_fn, cfg)
    if cfg.verbose and res is not None:
        print(res)
    return res


if __name__ == "__main__":
    main()
