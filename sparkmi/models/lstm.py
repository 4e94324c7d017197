"""LSTM text classifier — the reference model of distributed_lstm.py:110-135 / pytorch_lstm.py:94-119.

Same module names and parameter shapes (``embedding.weight``, ``lstm.weight_ih_l0`` ...
``lstm.bias_hh_l1``, ``fc_out.weight/bias``) so a reference state_dict loads unchanged, and the
same call contract ``forward(input_seq, hidden_in, mem_in) -> (pred [B,T,C], hidden_out,
mem_out)``.  The whole network (embedding gather, both LSTM layers with nn.LSTM's inter-layer
dropout, and the per-step fc head) runs as one persistent HIP kernel per direction on MI355X
(sparkmi/ops/lstm.py); ``nn.LSTM`` is only the parameter container.

Reference details kept: the embedding width is ``hidden_size`` (not ``embedding_dim``,
distributed_lstm.py:115), fc_out is ``Linear(hidden_size, output_size)`` (the reference hard-codes
32 == hidden_size, :122), ``padding_idx`` is the caller's (the reference passes ``vocab['0']``,
SURVEY Q10).  The sequential script's unused ``Dropout(0.5)`` (pytorch_lstm.py:109) is kept as an
attribute-free no-op.
"""
import torch
from torch import nn

from ..ops import rng as _rng
from ..ops.lstm import lstm_classifier, lstm_classifier_ce, lstm_classifier_last
from ..ops.loss import cross_entropy


class LSTM(nn.Module):
    def __init__(self, vocab_size, embedding_dim, hidden_size, output_size, num_layers=2, padding_idx=None,
                 dropout=0.5, seed=0, salt_base=1):
        super().__init__()
        self.embedding = nn.Embedding(num_embeddings=vocab_size, embedding_dim=hidden_size, padding_idx=padding_idx)
        self.lstm = nn.LSTM(input_size=embedding_dim, hidden_size=hidden_size, num_layers=num_layers,
                            batch_first=True, dropout=dropout)
        self.fc_out = nn.Linear(hidden_size, output_size)
        self.num_layers, self.hidden_size, self.dropout_p = num_layers, hidden_size, dropout
        self.padding_idx = padding_idx
        self.rng = _rng.DropoutRNG(seed)
        with _rng.salt_scope(salt_base):  # the model's own salt stream: masks independent of other models
            self.salt = _rng.new_salt()
        # ticket counters of the fused kernels (forward CE, embedding side plan, weight-gradient
        # column tiles; re-armed by the kernels): per model, so two models never share them; not
        # part of the state_dict (reference key parity).  One launch of a model at a time: LSTM
        # launches of ONE model on concurrent streams would share them.
        self.register_buffer("_tick", torch.zeros(48, dtype=torch.int32), persistent=False)
        self.last_ids = None

    def sparse_rows(self, cap=None):
        """{embedding weight: the last TRAINING batch's token ids}: its gradient touches only those
        rows (DataParallel(sparse_rows=...), the optional row-sparse exchange of SURVEY §5.8).  The
        ids are recorded only by a grad-enabled forward in training mode, so an evaluation pass
        between training steps (no_grad or eval()) cannot redirect the exchange to its rows.
        ``cap`` (e.g. batch * max sequence length): a fixed id-list capacity, no host sync."""
        fn = lambda: self.last_ids  # noqa: E731
        return {self.embedding.weight: (fn, int(cap)) if cap else fn}

    def _record_ids(self, input_seq):
        if self.training and torch.is_grad_enabled() and self.embedding.weight.requires_grad:
            self.last_ids = input_seq

    def param_list(self):
        ps = [self.embedding.weight]
        for i in range(self.num_layers):
            ps += [getattr(self.lstm, f"weight_ih_l{i}"), getattr(self.lstm, f"weight_hh_l{i}"),
                   getattr(self.lstm, f"bias_ih_l{i}"), getattr(self.lstm, f"bias_hh_l{i}")]
        return ps + [self.fc_out.weight, self.fc_out.bias]

    def init_state(self, batch_size, device=None):
        device = device or self.embedding.weight.device
        z = torch.zeros(self.num_layers, batch_size, self.hidden_size, device=device)
        return z, z.clone()

    def forward(self, input_seq, hidden_in=None, mem_in=None):
        self._record_ids(input_seq)
        return lstm_classifier(input_seq, hidden_in, mem_in, self.param_list(), self.num_layers,
                               dropout=self.dropout_p, training=self.training, rng=self.rng, salt=self.salt,
                               padding_idx=self.padding_idx, tick=self._tick)

    def loss(self, input_seq, labels, hidden_in=None, mem_in=None):
        """CE on the last step's prediction (distributed_lstm.py:186-189); returns (loss, pred)."""
        self._record_ids(input_seq)
        if (input_seq.is_cuda and labels.dim() == 1 and labels.is_cuda and labels.device == input_seq.device
                and labels.dtype in (torch.int64, torch.int32)):
            # GPU: the CE of the last step is fused into the LSTM forward kernel's tail (row loss,
            # head gradient, fixed-order mean through a ticket): no separate CE launches.  Class
            # ids must lie in [0, C) (the reference's labels - 1 of AG_NEWS, distributed_lstm.py:180;
            # no ignore_index): the kernel clamps an out-of-range id rather than read out of bounds
            return lstm_classifier_ce(input_seq, labels, hidden_in, mem_in, self.param_list(), self.num_layers,
                                      dropout=self.dropout_p, training=self.training, rng=self.rng, salt=self.salt,
                                      padding_idx=self.padding_idx, tick=self._tick)
        last, _, _, _ = lstm_classifier_last(input_seq, hidden_in, mem_in, self.param_list(), self.num_layers,
                                             dropout=self.dropout_p, training=self.training, rng=self.rng,
                                             salt=self.salt, padding_idx=self.padding_idx, tick=self._tick)
        # sparkmi's CE kernel (csrc/kernels/cross_entropy.hip: fixed-order loss sum) instead of the
        # ATen softmax / nll_loss launches; the CPU path falls back to the same math in torch
        return cross_entropy(last, labels), last


TextClassifierLSTM = LSTM
