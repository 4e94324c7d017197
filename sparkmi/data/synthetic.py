"""Synthetic datasets with the reference workloads' shapes (no network: the reference's
downloads — Spark's sample_multiclass_classification_data.txt, torchvision FashionMNIST,
torchtext AG_NEWS / Multi30k — are not available, SURVEY.md §0.1 finding 6).

All generators are deterministic in ``seed`` and can emit tensors directly on a device, so an
executor can keep its whole partition resident in HBM.
"""
import math

import numpy as np
import torch

SPECIALS = ["<pad>", "<sos>", "<eos>", "<unk>"]
PAD, SOS, EOS, UNK = 0, 1, 2, 3


def _gen(seed, device="cpu"):
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    return g


def iris_like(n=150, num_features=4, num_classes=3, seed=1234):
    """Iris-like 3-class 4-feature data (the shape of Spark's sample_multiclass_classification_data.txt:
    150 rows, features in [-1, 1], labels 0..2).  Returns (labels float64 [n], features float64 [n,F])."""
    rng = np.random.default_rng(seed)
    centers = rng.uniform(-0.6, 0.6, size=(num_classes, num_features))
    y = np.repeat(np.arange(num_classes), int(math.ceil(n / num_classes)))[:n]
    rng.shuffle(y)
    x = centers[y] + rng.normal(0, 0.18, size=(n, num_features))
    x = np.clip(x, -1.0, 1.0)
    return y.astype(np.float64), x


def iris_libsvm_text(n=150, num_features=4, num_classes=3, seed=1234, sparsify=True):
    """The iris-like data serialised in libsvm text format (1-based indices; zeros omitted)."""
    y, x = iris_like(n, num_features, num_classes, seed)
    lines = []
    for lab, row in zip(y, x):
        parts = [f"{int(lab)}"]
        for j, v in enumerate(row):
            if sparsify and abs(v) < 0.02:
                continue
            parts.append(f"{j + 1}:{v:.6f}")
        lines.append(" ".join(parts))
    return "\n".join(lines) + "\n"


def fashion_mnist_like(n=60000, seed=0, device="cpu", proto_seed=0):
    """uint8 images [n,1,28,28] and int64 labels [n] with class-dependent structure (10 classes),
    the shape of torchvision FashionMNIST (distributed_cnn.py:90-106).  The class prototypes come
    from ``proto_seed`` (shared by train and test splits), the samples from ``seed``."""
    proto = torch.rand(10, 1, 28, 28, generator=_gen(proto_seed + 7919, "cpu")).to(device)
    g = _gen(seed, device)
    labels = torch.randint(0, 10, (n,), generator=g, device=device)
    noise = torch.rand(n, 1, 28, 28, generator=g, device=device)
    img = (0.6 * proto[labels] + 0.4 * noise) * 255.0
    return img.to(torch.uint8), labels


def token_sequences(n, seq_len, vocab_size, min_len=None, seed=0, device="cpu", add_sos_eos=True):
    """Padded token-id sequences shaped like the reference text transforms' output:
    [<sos>, w..., <eos>, <pad>...] with w in [4, vocab) (distributed_lstm.py:96-107,
    pytorch_machine_translator.py:70-98).  Returns int64 [n, seq_len]."""
    g = _gen(seed, device)
    min_len = min_len or max(2, seq_len // 2)
    lengths = torch.randint(min_len, seq_len + 1, (n,), generator=g, device=device)
    ids = torch.randint(len(SPECIALS), vocab_size, (n, seq_len), generator=g, device=device)
    pos = torch.arange(seq_len, device=device)[None, :]
    if add_sos_eos:
        ids[:, 0] = SOS
        ids = torch.where(pos == (lengths[:, None] - 1), torch.full_like(ids, EOS), ids)
    ids = torch.where(pos >= lengths[:, None], torch.full_like(ids, PAD), ids)
    return ids


def translation_pairs(n, seq_len, src_vocab, tgt_vocab, seed=0, device="cpu"):
    """Multi30k-like parallel corpus as padded id tensors (src [n,S], tgt [n,S])."""
    return (token_sequences(n, seq_len, src_vocab, seed=seed, device=device),
            token_sequences(n, seq_len, tgt_vocab, seed=seed + 1, device=device))


def copy_pairs(n, seq_len, vocab, seed=0, device="cpu"):
    """A LEARNABLE parallel corpus of the same shape: tgt = a fixed permutation of the source
    tokens (same lengths and specials).  ``translation_pairs`` draws src and tgt independently
    and uniformly, so no model can beat the token entropy there (cross-entropy floor ln(vocab - 4),
    9.21 at vocab 10000); here the loss can fall to zero."""
    src = token_sequences(n, seq_len, vocab, seed=seed, device=device)
    g = _gen(seed + 11, device)
    perm = torch.arange(vocab, device=device)
    perm[len(SPECIALS):] = len(SPECIALS) + torch.randperm(vocab - len(SPECIALS), generator=g, device=device)
    return src, perm[src]


def ag_news_like(n, seq_len, vocab_size, num_classes=4, seed=0, device="cpu"):
    """AG_NEWS-like classification: padded ids [n, seq_len] and labels [n] in 0..3 where the label
    is weakly encoded in the token distribution (so training makes progress)."""
    g = _gen(seed, device)
    labels = torch.randint(0, num_classes, (n,), generator=g, device=device)
    ids = token_sequences(n, seq_len, vocab_size, seed=seed + 7, device=device)
    # plant class-indicative tokens
    marker = 4 + labels * 3
    pos = torch.randint(1, max(2, seq_len // 2), (n,), generator=g, device=device)
    ids[torch.arange(n, device=device), pos] = marker
    return ids, labels


_WORDS = ("a man woman child dog cat plays runs walks sits street park water ball red blue green small large "
          "young old group people two three in on at with the of and is are near while holding wearing").split()


def sentences(n, min_words=4, max_words=14, seed=0):
    """Random English-like sentences (for tokenizer / vocab / text-pipeline tests)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        k = int(rng.integers(min_words, max_words + 1))
        words = [_WORDS[int(i)] for i in rng.integers(0, len(_WORDS), size=k)]
        s = " ".join(words).capitalize()
        if rng.random() < 0.3:
            s += ","
        out.append(s + rng.choice([".", "!", "?"]))
    return out


_TOPICS = {
    1: "world government minister election president war peace talks country leaders capital".split(),
    2: "sports game team season coach player win championship league score match".split(),
    3: "business market stocks company profit shares oil prices economy deal bank".split(),
    4: "technology software internet computer space research science phone web data".split(),
}


def ag_news_text(n, seed=0, min_words=8, max_words=60):
    """AG_NEWS-like (label, text) pairs with labels 1..4 (torchtext AG_NEWS yields 1-based labels,
    distributed_lstm.py:180 subtracts 1).  Each text mixes topic words with filler words and
    numbers, so basic_english tokenisation, vocab building and the <sos>/<eos>/truncate/pad
    transforms are exercised on realistic strings."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        lab = int(rng.integers(1, 5))
        k = int(rng.integers(min_words, max_words + 1))
        topic = _TOPICS[lab]
        words = []
        for _ in range(k):
            r = rng.random()
            if r < 0.35:
                words.append(topic[int(rng.integers(0, len(topic)))])
            elif r < 0.45:
                words.append(str(int(rng.integers(0, 100))))
            else:
                words.append(_WORDS[int(rng.integers(0, len(_WORDS)))])
        text = " ".join(words).capitalize() + rng.choice([".", "!", "?", " (AP)"])
        out.append((lab, text))
    return out


def _pseudo_de(word):
    return (word[::-1] + "en") if word.isalpha() else word


def translation_text(n, seed=0, min_words=4, max_words=14):
    """Multi30k-like parallel corpus of (english, pseudo-german) sentence pairs; the German side
    is a deterministic word-level mapping of the English side, so a translator can learn it
    (pytorch_machine_translator.py:14-16 reads Multi30k, unavailable offline)."""
    out = []
    for s in sentences(n, min_words, max_words, seed):
        words = s.split(" ")
        de = " ".join(_pseudo_de(w.lower().strip(".,!?")) for w in words) + s[-1]
        out.append((s, de.capitalize()))
    return out
