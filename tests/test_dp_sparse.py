"""Row-sparse exchange of the LSTM embedding gradient (the embedding of
/root/reference/distributed_lstm.py:115) on CPU with gloo, 2 real processes:

* DataParallel(sparse_rows=...) gives the parameters of the dense all-reduce after several Adam
  steps (the reconstructed dense gradient has zeros exactly where the all-reduced one does, so
  Adam's decay of untouched rows is unchanged), while moving far fewer bytes;
* rows touched by both ranks and repeated ids within a rank are summed once per occurrence
  (the embedding backward already summed them locally; the exchange de-duplicates the ids).
"""
import sys

import cloudpickle
import torch

from sparkmi.api import Distributor

cloudpickle.register_pickle_by_value(sys.modules[__name__])

V, T, B = 300, 12, 4


def _run(steps, sparse, cap=None, eval_between=False):
    import torch
    from sparkmi.models.lstm import LSTM
    from sparkmi.optim import Adam
    from sparkmi.parallel import DataParallel, init_distributed, rank, world_size
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    init_distributed()
    torch.manual_seed(4)
    m = LSTM(V, 32, 32, 4, num_layers=2, padding_idx=0, dropout=0.0).train()
    flat = FlatParams(m)
    opt = Adam(flat, lr=1e-2)
    ws, r = world_size(), rank()
    ddp = DataParallel(flat, bucket_mb=0.05, sparse_rows=m.sparse_rows(cap=cap) if sparse else None)
    runner = StepRunner(m, lambda mm, x, y: mm.loss(x, y)[0], opt, ddp, graph=False)
    g = torch.Generator().manual_seed(11)
    # a small id range so both ranks touch common rows and repeat ids within a batch
    ids = torch.randint(1, 40, (steps, 2 * B, T), generator=g)
    ids[:, :, -2:] = 0  # padding tokens
    lbl = torch.randint(0, 4, (steps, 2 * B), generator=g)
    for i in range(steps):
        runner.step(ids[i, r * B:(r + 1) * B], lbl[i, r * B:(r + 1) * B])
        if eval_between:  # a validation pass between steps must not redirect the exchange
            with torch.no_grad():
                m(torch.randint(50, V, (B, T), generator=g))
            m.eval()
            m.loss(torch.randint(50, V, (B, T), generator=g), lbl[i, :B])
            m.train()
    out = (flat.master.clone(), ddp.bytes_reduced)
    ddp.close()
    return out


def _dp(sparse, steps=3, cap=None, eval_between=False):
    return Distributor(num_processes=2, use_gpu=False, log_sink=None, timeout=300).run(_run, steps, sparse, cap,
                                                                                          eval_between)


def test_sparse_embedding_exchange_matches_dense_allreduce():
    dense, dense_bytes = _dp(False)
    sparse, sparse_bytes = _dp(True)
    assert torch.allclose(sparse, dense, rtol=1e-6, atol=1e-7), float((sparse - dense).abs().max())
    # the 300 x 32 table: 38,400 B dense per step vs B*T = 48 ids x (8 + 128) B = 6,528 B
    assert sparse_bytes < dense_bytes - 3 * (V * 32 * 4 - B * T * 136) + 1


def test_sparse_exchange_fixed_capacity_and_eval_between_steps():
    """A fixed id-list capacity (no host sync) gives the same parameters, and evaluation forwards
    between the training steps (no_grad, eval mode) do not change which rows are exchanged
    (the ids are recorded by grad-enabled training forwards only)."""
    dense, _ = _dp(False, eval_between=True)
    capped, _ = _dp(True, cap=B * T + 7, eval_between=True)
    assert torch.allclose(capped, dense, rtol=1e-6, atol=1e-7), float((capped - dense).abs().max())


def _run_over(cap):
    """Rank 0 alone exceeds the fixed capacity; both ranks must still complete the exchange and
    then raise together at check().  Returns every rank's outcome (gathered to rank 0)."""
    import torch
    import torch.distributed as dist
    from sparkmi.models.lstm import LSTM
    from sparkmi.optim import Adam
    from sparkmi.parallel import DataParallel, init_distributed, rank
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    init_distributed()
    torch.manual_seed(4)
    m = LSTM(V, 32, 32, 4, num_layers=2, padding_idx=0, dropout=0.0).train()
    flat = FlatParams(m)
    ddp = DataParallel(flat, bucket_mb=0.05, sparse_rows=m.sparse_rows(cap=cap))
    runner = StepRunner(m, lambda mm, x, y: mm.loss(x, y)[0], Adam(flat, lr=1e-2), ddp, graph=False)
    r = rank()
    hi = 120 if r == 0 else 3  # rank 0: many distinct ids; rank 1: ids 1-2 only (under the cap)
    g = torch.Generator().manual_seed(5 + r)
    runner.step(torch.randint(1, hi, (B, T), generator=g), torch.randint(0, 4, (B,), generator=g))
    try:
        ddp.check()
        out = "ok"
    except ValueError as e:
        out = "raised: " + str(e)[:40]
    outs = [None, None]
    dist.all_gather_object(outs, out)
    ddp.close()
    return outs


def test_sparse_capacity_overflow_raises_on_every_rank():
    """a rank whose unique ids exceed the fixed capacity used to raise BEFORE the
    all-gather and leave its peer blocked in it; now the overflow travels as a flag slot of the
    gathered id list and check() raises on every rank."""
    outs = Distributor(num_processes=2, use_gpu=False, log_sink=None, timeout=300).run(_run_over, 8)
    assert all(o.startswith("raised") for o in outs), outs
