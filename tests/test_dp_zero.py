"""T2 data-parallel engine on CPU (gloo, 2 real processes):

* ZeRO-1 (reduce-scatter -> sharded multi-range Adam -> in-place all-gather) gives the SAME
  parameters, bit for bit, as plain all-reduce data parallelism, through StepRunner, with the
  split (multi-piece) backward and its bucket re-cut + moment re-shard, and with small buckets;
* transformer data parallelism: 2 ranks x batch b == 1 rank x batch 2b (same global batch),
  params after several Adam steps agree to fp32 reassociation tolerance;
* optimizer per bucket: each bucket's Adam update right after its own reduction equals the
  single update bit for bit (plain and ZeRO-1);
* per-bucket early flush: with deferred (grouped) weight gradients, buckets still complete
  during the backward (DataParallel.early_flushes) and the result equals the non-deferred run.
Reference collective sites: distributed_multilayer_perceptron.py:103-106,
distributed_cnn.py:152-156 (DDP intended but never synchronising).
"""
import sys

import cloudpickle
import pytest
import torch

from sparkmi.api import Distributor

cloudpickle.register_pickle_by_value(sys.modules[__name__])

V, S, B = 48, 16, 4


def _data(steps, batch, seed=7):
    g = torch.Generator().manual_seed(seed)
    # no pad tokens (id 0): every rank's masked-mean CE has the same token count, so the
    # average of per-rank means equals the global mean exactly as in the single-rank run
    src = torch.randint(1, V, (steps, batch, S), generator=g)
    tgt = torch.randint(1, V, (steps, batch, S), generator=g)
    return src, tgt


def _make(seed=3):
    from sparkmi.models.transformer import Transformer
    torch.manual_seed(seed)
    m = Transformer(d_model=64, ffn_hidden=128, num_heads=1, num_layers=2, max_sequence_length=S,
                    src_vocab_size=V, tgt_vocab_size=V, drop_prob=0.0, emb_dropout=0.0, seed=1)
    return m.train()


def _run(steps, zero, split, bucket_mb, dp=True, global_batch=2 * B, per_bucket=None):
    import torch
    from sparkmi.optim import Adam
    from sparkmi.parallel import DataParallel, init_distributed, rank, world_size
    from sparkmi.parallel import ddp as ddp_mod
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    init_distributed()
    if per_bucket is not None:
        ddp_mod.PER_BUCKET_OPT = per_bucket
    m = _make()
    flat = FlatParams(m)
    opt = Adam(flat, lr=1e-2)
    ws, r = world_size(), rank()
    ddp = DataParallel(flat, bucket_mb=bucket_mb, zero=zero) if (dp and ws > 1) else None
    split_fn = (lambda mm, s, t: mm.training_step_split(s, t)) if split else None
    runner = StepRunner(m, lambda mm, s, t: mm.training_step_loss(s, t), opt, ddp, graph=False, split_fn=split_fn)
    src, tgt = _data(steps, global_batch)
    per = global_batch // ws
    for i in range(steps):
        runner.step(src[i, r * per:(r + 1) * per], tgt[i, r * per:(r + 1) * per])
    out = flat.master.clone()
    if ddp is not None:
        ddp.close()
        if per_bucket is not None:
            return out, ddp.opt_buckets_early, len(ddp.buckets)
    return out


def _dp(zero, split=False, bucket_mb=0.25, steps=4, per_bucket=None):
    return Distributor(num_processes=2, use_gpu=False, log_sink=None, timeout=300).run(
        _run, steps, zero, split, bucket_mb, per_bucket=per_bucket)


def test_zero1_equals_allreduce_bitwise():
    a = _dp(False)
    b = _dp(True)
    assert torch.equal(a, b)


def test_zero1_split_backward_reshard_bitwise():
    a = _dp(False, split=True)
    b = _dp(True, split=True)
    assert torch.equal(a, b)


@pytest.mark.parametrize("zero,split", [(False, False), (True, False), (True, True)])
def test_per_bucket_optimizer_bitwise(zero, split):
    """the Adam update per gradient bucket, each behind its own
    reduction (DataParallel.attach_optimizer), gives the one-update-after-all-buckets parameters bit
    for bit — plain all-reduce and ZeRO-1 (owned pieces, compact moments), with the split backward's
    bucket re-cut and moment re-shard; every bucket but the last is updated early."""
    a, na, nb = _dp(zero, split=split, bucket_mb=0.05, per_bucket=True)
    b, nb0, _ = _dp(zero, split=split, bucket_mb=0.05, per_bucket=False)
    assert nb > 2 and na == nb - 1 and nb0 == 0
    assert torch.equal(a, b)


def _grads(split):
    """One backward: the averaged data-parallel gradient (or the single-rank one)."""
    import torch
    from sparkmi.optim import Adam
    from sparkmi.parallel import DataParallel, init_distributed, rank, world_size
    from sparkmi.utils.flat import FlatParams
    init_distributed()
    m = _make()
    flat = FlatParams(m)
    ws, r = world_size(), rank()
    ddp = DataParallel(flat, bucket_mb=0.25) if ws > 1 else None
    src, tgt = _data(1, 2 * B)
    per = 2 * B // ws
    loss = m.training_step_loss(src[0, r * per:(r + 1) * per], tgt[0, r * per:(r + 1) * per])
    loss.backward()
    if ddp is not None:
        ddp.finish()
        ddp.close()
    return flat.grad / ws


def test_transformer_dp_gradient_matches_single_rank_large_batch():
    dp = Distributor(num_processes=2, use_gpu=False, log_sink=None, timeout=300).run(_grads, False)
    single = _grads(False)
    torch.testing.assert_close(dp, single, atol=1e-6, rtol=1e-4)


def test_transformer_dp_matches_single_rank_large_batch():
    """Several Adam steps: trajectories agree up to fp32 reassociation (Adam's m/sqrt(v) turns
    ~1e-8 gradient differences on near-zero gradients into lr-sized ones, so a handful of
    elements move; the parameter vector as a whole stays on the single-rank trajectory)."""
    dp = _dp(False, steps=3)
    single = _run(3, False, False, 0.25, dp=False)
    assert float((dp - single).norm() / single.norm()) < 1e-4
    assert float((dp - single).abs().gt(1e-5).float().mean()) < 0.01


def _early(steps):
    import torch
    from sparkmi.optim import Adam
    from sparkmi.parallel import DataParallel, init_distributed, rank
    from sparkmi.utils.flat import FlatParams
    from sparkmi.ops import _grad
    init_distributed()
    m = _make()
    flat = FlatParams(m)
    opt = Adam(flat, lr=1e-2)
    ddp = DataParallel(flat, bucket_mb=0.05)
    opt.grad_scale = ddp.grad_scale
    src, tgt = _data(steps, 2 * B)
    r = rank()
    flushes = 0
    for i in range(steps):
        loss = m.training_step_loss(src[i, r * B:(r + 1) * B], tgt[i, r * B:(r + 1) * B])
        loss.backward()
        assert not _grad.pending()
        ddp.finish()
        opt.step()
    ddp.close()
    return flat.master.clone()


def test_dp_eager_overlap_listener_equivalent():
    a = Distributor(num_processes=2, use_gpu=False, log_sink=None, timeout=300).run(_early, 3)
    b = _dp(False, steps=3, bucket_mb=0.05)
    torch.testing.assert_close(a, b, atol=0, rtol=0)


def test_deferred_queue_recovers_after_failed_backward():
    """ADVICE: a backward that raises after queueing deferred work must not poison later steps."""
    from sparkmi.ops import _grad
    _grad._ln_queue.append(("stale",))
    _grad._cb[0] = True
    assert _grad.reset_deferred() is True
    assert not _grad.pending()


def test_ipc_capacity_covers_oversized_parameter_buckets():
    """a parameter larger than the bucket limit gets a bucket of its own that exceeds
    the limit; the IPC staging capacity must cover it (and every re-cut by align_buckets)."""
    from sparkmi.parallel.ddp import DataParallel
    from sparkmi.utils.flat import FlatParams
    m = torch.nn.Sequential(torch.nn.Embedding(5000, 32), torch.nn.Linear(32, 4))  # 160k-float embedding
    flat = FlatParams(m, device="cpu", shadow=False)
    dp = DataParallel.__new__(DataParallel)
    dp.flat, dp._limit = flat, 1000          # bucket limit far below the embedding
    dp._build_buckets()
    cap = dp._ipc_capacity()
    assert max(e - s for s, e, _ in dp.buckets) <= cap
    for cuts in ([1], [1, 2], [0, 1, 2]):
        dp._build_buckets(cuts)
        assert max(e - s for s, e, _ in dp.buckets) <= cap
    assert cap >= 5000 * 32


def test_choose_comm_prefers_the_measured_faster_path():
    """Bulk-gradient path selection from the start-up measurement."""
    from sparkmi.parallel.ddp import choose_comm
    assert choose_comm(1.0, 2.0) == "ipc"
    assert choose_comm(2.0, 1.0) == "rccl"
    assert choose_comm(1.5, 1.5) == "ipc"        # a tie keeps the graph-capturable kernel
    assert choose_comm(None, 1.0) == "rccl"      # IPC unavailable
    assert choose_comm(1.0, None) == "ipc"


def test_dp_probe_disabled_uses_rccl_for_bulk(monkeypatch):
    """SPARKMI_DP_PROBE=0: a bulk gradient (> IPC_LIMIT_BYTES) goes to the process group without
    building the IPC path; world 1 never probes."""
    from sparkmi.parallel import ddp
    from sparkmi.utils.flat import FlatParams
    monkeypatch.setenv("SPARKMI_DP_PROBE", "0")
    monkeypatch.setattr(ddp, "IPC_LIMIT_BYTES", 16)
    flat = FlatParams(torch.nn.Linear(8, 8), device="cpu", shadow=False)
    dp = ddp.DataParallel(flat)
    assert dp.ipc is None and dp.comm_probe is None and dp.comm == "none"


def test_choose_comm_three_paths():
    """The probe's three candidates: IPC two-shot, the default RCCL
    communicator and the min_ctas multi-channel one; fastest wins, ties prefer that order."""
    from sparkmi.parallel.ddp import choose_comm
    assert choose_comm(3.0, 2.0, 1.0) == "rccl_mc"
    assert choose_comm(1.0, 2.0, 1.0) == "ipc"
    assert choose_comm(None, 2.0, 2.0) == "rccl"
    assert choose_comm(None, 2.0, 1.5) == "rccl_mc"
    assert choose_comm(None, None, None) == "rccl"
    assert choose_comm(None, 2.0, None) == "rccl"


def test_choose_comm_four_paths():
    """the zero-copy IPC two-shot is a fourth probed candidate — fastest wins; ties
    prefer staged IPC, then zero-copy IPC, then the RCCL groups; a candidate that failed its exact-
    sum / timeout check (None) is never chosen."""
    from sparkmi.parallel.ddp import choose_comm
    assert choose_comm(2.0, 3.0, 3.0, 1.0) == "ipc_zc"
    assert choose_comm(1.0, 3.0, 3.0, 1.0) == "ipc"        # tie: the staged kernel
    assert choose_comm(None, 3.0, 3.0, 2.0) == "ipc_zc"
    assert choose_comm(2.0, 1.0, 3.0, 1.0) == "ipc_zc"     # tie with rccl: the graph-capturable kernel
    assert choose_comm(2.0, 1.0, 0.5, 1.5) == "rccl_mc"
    assert choose_comm(2.0, 1.0, None, None) == "rccl"
    assert choose_comm(None, None, None, None) == "rccl"
    assert choose_comm(None, 2.0, None, 0.1) == "ipc_zc"


def _probe_run():
    import torch
    from sparkmi.parallel import ddp, init_distributed
    from sparkmi.utils.flat import FlatParams
    init_distributed()
    ddp.IPC_LIMIT_BYTES = 1024  # a "bulk" gradient at test size
    flat = FlatParams(torch.nn.Linear(64, 64), device="cpu", shadow=False)
    dp = ddp.DataParallel(flat)
    out = (dp.comm_probe, dp.comm, dp.bulk_group is None)
    dp.close()
    return out


def test_dp_probe_lists_three_paths_gloo():
    """Two CPU ranks over gloo: the start-up probe measures the process group, reports the IPC and
    multi-channel RCCL candidates as unavailable (None) and keeps the default group."""
    from sparkmi.api import Distributor
    probe, comm, default_group = Distributor(num_processes=2, use_gpu=False, log_sink=None,
                                             timeout=120).run(_probe_run)
    assert set(probe) >= {"bucket_bytes", "ipc_ms", "ipc_zc_ms", "rccl_ms", "rccl_min_ctas32_ms", "choice"}
    assert probe["ipc_ms"] is None and probe["ipc_zc_ms"] is None and probe["rccl_min_ctas32_ms"] is None
    assert probe["rccl_ms"] > 0
    assert probe["choice"] == "rccl" and comm == "rccl" and default_group
