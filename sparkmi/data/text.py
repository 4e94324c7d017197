"""Text pipeline: torchtext-compatible basic_english tokenizer, specials-first Vocab, and the
VocabTransform -> AddToken(sos) -> Truncate -> AddToken(eos) -> ToTensor(pad) -> PadTransform
chain (distributed_lstm.py:75-107, pytorch_machine_translator.py:20-98).

The tokenizer, vocabulary build and the fused batch encoder are C++ (csrc/runtime/text.cpp,
sparkmi._runtime); this module gives them the torchtext-shaped Python surface
(``get_tokenizer``, ``build_vocab_from_iterator``, ``transforms.Sequential`` ...).  A pure-Python
``basic_english_py`` is kept as the executable spec the C++ tokenizer is tested against.
"""
import re
from collections import Counter

import torch

from .. import _native

SPECIALS = ["<pad>", "<sos>", "<eos>", "<unk>"]

_PATTERNS = [(re.compile(p), r) for p, r in [
    (r"\'", " '  "), (r"\"", ""), (r"\.", " . "), (r"<br \/>", " "), (r",", " , "), (r"\(", " ( "), (r"\)", " ) "),
    (r"\!", " ! "), (r"\?", " ? "), (r"\;", " "), (r"\:", " "), (r"\s+", " ")]]


def basic_english_py(line: str):
    """Reference (pure Python) basic_english normalisation + whitespace split."""
    line = line.lower()
    for pat, rep in _PATTERNS:
        line = pat.sub(rep, line)
    return line.split()


def get_tokenizer(name="basic_english", language=None):
    """torchtext.data.utils.get_tokenizer.  'basic_english' runs in C++; 'spacy' is not
    available offline and falls back to a whitespace/punctuation tokenizer."""
    if name == "basic_english":
        rt = _native.RT()
        return rt.tokenize_basic_english
    if name in ("spacy", "whitespace", None):
        rt = _native.RT()
        return rt.tokenize_basic_english
    if callable(name):
        return name
    raise ValueError(f"unknown tokenizer {name}")


class Vocab:
    """torchtext.vocab.Vocab-compatible wrapper over the C++ vocabulary."""

    def __init__(self, cpp):
        self._v = cpp

    def __len__(self):
        return len(self._v)

    def __getitem__(self, token):
        return self._v[token]

    def __contains__(self, token):
        return token in self._v

    def set_default_index(self, index):
        self._v.set_default_index(int(index))

    def get_default_index(self):
        i = self._v.get_default_index()
        return None if i < 0 else i

    def get_itos(self):
        return self._v.get_itos()

    def get_stoi(self):
        return {t: i for i, t in enumerate(self._v.get_itos())}

    def lookup_indices(self, tokens):
        return self._v.lookup_indices(list(tokens))

    def lookup_token(self, index):
        return self._v.get_itos()[index]

    def __call__(self, tokens):
        return self.lookup_indices(tokens)

    def encode_batch(self, token_lists, sos=-1, eos=-1, max_len=0, pad=0, pad_to=0):
        return torch.from_numpy(self._v.encode_batch(token_lists, sos, eos, max_len, pad, pad_to))


def build_vocab_from_iterator(iterator, min_freq=1, specials=None, special_first=True):
    """torchtext semantics: specials first (ids 0..), then tokens by descending frequency, ties by
    token order; tokens below min_freq dropped."""
    counts = Counter()
    for toks in iterator:
        counts.update(toks)
    rt = _native.RT()
    return Vocab(rt.Vocab.build(dict(counts), int(min_freq), list(specials or []), bool(special_first)))


def build_vocab_from_texts(texts, min_freq=1, specials=SPECIALS, special_first=True):
    """Fast path: tokenize + count in C++."""
    rt = _native.RT()
    counts = rt.count_tokens(list(texts))
    return Vocab(rt.Vocab.build(counts, int(min_freq), list(specials or []), bool(special_first)))


class transforms:
    """torchtext.transforms subset; ``Sequential`` of the standard chain collapses into one C++ call."""

    class VocabTransform:
        def __init__(self, vocab):
            self.vocab = vocab

        def __call__(self, batch):
            return [self.vocab.lookup_indices(t) for t in batch]

    class AddToken:
        def __init__(self, token, begin=True):
            self.token, self.begin = token, begin

        def __call__(self, batch):
            return [([self.token] + list(x)) if self.begin else (list(x) + [self.token]) for x in batch]

    class Truncate:
        def __init__(self, max_seq_len):
            self.max_seq_len = max_seq_len

        def __call__(self, batch):
            return [list(x)[:self.max_seq_len] for x in batch]

    class ToTensor:
        def __init__(self, padding_value=0, dtype=torch.long):
            self.padding_value, self.dtype = padding_value, dtype

        def __call__(self, batch):
            L = max((len(x) for x in batch), default=0)
            out = torch.full((len(batch), L), self.padding_value, dtype=self.dtype)
            for i, x in enumerate(batch):
                out[i, :len(x)] = torch.as_tensor(list(x), dtype=self.dtype)
            return out

    class PadTransform:
        def __init__(self, max_length, pad_value):
            self.max_length, self.pad_value = max_length, pad_value

        def __call__(self, x):
            if x.shape[-1] >= self.max_length:
                return x
            pad = torch.full((*x.shape[:-1], self.max_length - x.shape[-1]), self.pad_value, dtype=x.dtype)
            return torch.cat([x, pad], dim=-1)

    class Sequential:
        def __init__(self, *steps):
            self.steps = list(steps)
            self._fast = self._plan()

        def _plan(self):
            """Recognise [Vocab, AddToken(begin), Truncate, AddToken(end), ToTensor, (PadTransform)]."""
            s = self.steps
            T = transforms
            if len(s) in (5, 6) and isinstance(s[0], T.VocabTransform) and isinstance(s[1], T.AddToken) and \
                    s[1].begin and isinstance(s[2], T.Truncate) and isinstance(s[3], T.AddToken) and \
                    not s[3].begin and isinstance(s[4], T.ToTensor) and \
                    (len(s) == 5 or isinstance(s[5], T.PadTransform)):
                pad_to = s[5].max_length if len(s) == 6 else 0
                return dict(vocab=s[0].vocab, sos=s[1].token, max_len=s[2].max_seq_len, eos=s[3].token,
                            pad=s[4].padding_value, pad_to=pad_to)
            return None

        def __call__(self, batch):
            if self._fast is not None:
                f = self._fast
                out = f["vocab"].encode_batch(batch, f["sos"], f["eos"], f["max_len"], f["pad"], 0)
                if f["pad_to"] and out.shape[1] < f["pad_to"]:
                    out = transforms.PadTransform(f["pad_to"], self.steps[5].pad_value)(out)
                return out
            x = batch
            for st in self.steps:
                x = st(x)
            return x


def text_pipeline(vocab, sos=1, eos=2, max_len=128, pad=0, pad_to=0):
    """The reference's transform chain as one callable (tokens -> padded int64 tensor)."""
    T = transforms
    steps = [T.VocabTransform(vocab), T.AddToken(sos, begin=True), T.Truncate(max_len), T.AddToken(eos, begin=False),
             T.ToTensor(padding_value=pad)]
    if pad_to:
        steps.append(T.PadTransform(pad_to, pad))
    return T.Sequential(*steps)
