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

    def sparse_rows(self):
        """{embedding weight: the last batch's token ids}: its gradient touches only those rows
        (DataParallel(sparse_rows=...), the optional row-sparse exchange of SURVEY §5.8)."""
        return {self.embedding.weight: lambda: self.last_ids}

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
        self.last_ids = input_seq
        return lstm_classifier(input_seq, hidden_in, mem_in, self.param_list(), self.num_layers,
                               dropout=self.dropout_p, training=self.training, rng=self.rng, salt=self.salt,
                               padding_idx=self.padding_idx)

    def loss(self, input_seq, labels, hidden_in=None, mem_in=None):
        """CE on the last step's prediction (distributed_lstm.py:186-189); returns (loss, pred)."""
        self.last_ids = input_seq
        if input_seq.is_cuda and labels.dim() == 1:
            # GPU: the CE of the last step is fused into the LSTM forward kernel's tail (row loss,
            # head gradient, fixed-order mean through a ticket): no separate CE launches
            return lstm_classifier_ce(input_seq, labels, hidden_in, mem_in, self.param_list(), self.num_layers,
                                      dropout=self.dropout_p, training=self.training, rng=self.rng, salt=self.salt,
                                      padding_idx=self.padding_idx)
        last, _, _, _ = lstm_classifier_last(input_seq, hidden_in, mem_in, self.param_list(), self.num_layers,
                                             dropout=self.dropout_p, training=self.training, rng=self.rng,
                                             salt=self.salt, padding_idx=self.padding_idx)
        # sparkmi's CE kernel (csrc/kernels/cross_entropy.hip: fixed-order loss sum) instead of the
        # ATen softmax / nll_loss launches; the CPU path falls back to the same math in torch
        return cross_entropy(last, labels), last


TextClassifierLSTM = LSTM
