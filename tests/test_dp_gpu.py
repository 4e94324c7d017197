"""Data-parallel step runner on the GPU: HIP-graph-captured forward+backward, then the bucketed
gradient all-reduce and the fused optimizer outside the graph.  Two executor processes share
the box's one MI355X and talk over gloo here (RCCL needs one device per rank); the code path
under test — capture with the overlap listener off, replay, finish(), optimizer — is the one
the multi-GPU RCCL run takes."""
import sys

import cloudpickle
import pytest
import torch

from sparkmi.runtime.launcher import launch

cloudpickle.register_pickle_by_value(sys.modules[__name__])


def _train(graph, steps, split=False):
    import torch
    import torch.distributed as dist
    from sparkmi.models.transformer import Transformer
    from sparkmi.optim import SGD
    from sparkmi.parallel import DataParallel, init_distributed
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    rank, world, device = init_distributed()
    torch.manual_seed(0)
    m = Transformer(d_model=128, ffn_hidden=256, num_heads=2, drop_prob=0.0, num_layers=2, max_sequence_length=64,
                    src_vocab_size=300, tgt_vocab_size=300, emb_dropout=0.0).to(device)
    flat = FlatParams(m)
    opt = SGD(flat, lr=0.05)  # linear in the gradients: no amplification of last-bit noise
    ddp = DataParallel(flat, bucket_mb=0.5)
    split_fn = (lambda mm, s, t: mm.training_step_split(s, t)) if split else None
    runner = StepRunner(m, lambda mm, s, t: mm.training_step_loss(s, t), opt, ddp, graph=graph, warmup_eager=2,
                        split_fn=split_fn)
    g = torch.Generator().manual_seed(1)
    data = torch.randint(4, 300, (steps, 2, 8, 64), generator=g).to(device)
    for i in range(steps):
        runner.step(data[i, 0, rank * 4:(rank + 1) * 4].contiguous(), data[i, 1, rank * 4:(rank + 1) * 4].contiguous())
    torch.cuda.synchronize()
    p = flat.master.clone()
    ref = p.clone()
    dist.broadcast(ref, 0)
    synced = bool(torch.equal(ref, p))
    info = ([len(w) for w in runner.bucket_waves], len(ddp.buckets)) if split else None
    return p.cpu(), synced, info


@pytest.mark.gpu
def test_graph_dp_matches_eager_dp():
    env = {"SPARKMI_DIST_BACKEND": "gloo"}
    pg, sg, _ = launch(_train, (True, 6), {}, num_processes=2, use_gpu=True, env=env, log_sink=None, timeout=300)
    pe, se, _ = launch(_train, (False, 6), {}, num_processes=2, use_gpu=True, env=env, log_sink=None, timeout=300)
    assert sg and se
    torch.testing.assert_close(pg, pe, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_split_graph_dp_matches_eager_dp():
    """Three-graph step (decoder backward, upper-encoder backward, lower-encoder backward, with
    each piece's final buckets all-reduced while the next runs) == eager DP."""
    env = {"SPARKMI_DIST_BACKEND": "gloo"}
    ps, ss, info = launch(_train, (True, 6, True), {}, num_processes=2, use_gpu=True, env=env, log_sink=None,
                          timeout=300)
    pe, se, _ = launch(_train, (False, 6), {}, num_processes=2, use_gpu=True, env=env, log_sink=None, timeout=300)
    assert ss and se
    waves, total = info
    assert len(waves) == 3 and all(w > 0 for w in waves[:2]) and sum(waves) <= total, info
    torch.testing.assert_close(ps, pe, rtol=1e-4, atol=1e-5)
