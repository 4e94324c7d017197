"""T2 CPU-distributed tests (gloo, real processes): the Distributor launcher contract, rank-0
result return, log streaming, failure propagation / restart, hang detection, the gradient-sync
regression for SURVEY Q1 (grads identical on every rank after backward), and DP parity (DP over
2 ranks at batch b == 1 rank at batch 2b)."""
import os
import sys

import cloudpickle
import pytest
import torch

from sparkmi.api import Distributor
from sparkmi.runtime import LaunchError

cloudpickle.register_pickle_by_value(sys.modules[__name__])


def _env_fn(x):
    import os
    return {k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}, x * 2


def test_run_returns_rank0_result():
    env, v = Distributor(num_processes=2, use_gpu=False).run(_env_fn, 21)
    assert v == 42
    assert env["RANK"] == "0" and env["WORLD_SIZE"] == "2" and env["MASTER_ADDR"] == "127.0.0.1"


def _print_fn():
    import os
    print("hello from", os.environ["RANK"], flush=True)
    return os.environ["RANK"]


def test_log_streaming():
    lines = []
    r = Distributor(num_processes=2, use_gpu=False, log_sink=lines.append).run(_print_fn)
    assert r == "0"
    assert any(l.startswith("[rank 1] hello from 1") for l in lines)


def _fail_fn():
    import os
    if os.environ["RANK"] == "1":
        raise ValueError("boom")
    import time
    time.sleep(60)


def test_failure_terminates_group():
    lines = []
    with pytest.raises(LaunchError) as e:
        Distributor(num_processes=2, use_gpu=False, log_sink=lines.append, timeout=120).run(_fail_fn)
    assert e.value.rank == 1
    assert "boom" in e.value.log_tail


def _restart_fn():
    import os
    from sparkmi.runtime import fault_point
    for step in range(3):
        fault_point(step)
    return int(os.environ["TORCHELASTIC_RESTART_COUNT"])


def test_restart_after_injected_fault():
    d = Distributor(num_processes=2, use_gpu=False, max_restarts=1, env={"SPARKMI_FAULT": "1:1:exit:0"},
                    log_sink=None)
    assert d.run(_restart_fn) == 1


def _hang_fn():
    from sparkmi.runtime import fault_point
    fault_point(0)


def test_hang_detected_by_heartbeat():
    d = Distributor(num_processes=2, use_gpu=False, heartbeat_timeout=3.0, env={"SPARKMI_FAULT": "0:0:hang",
                    "SPARKMI_HEARTBEAT_PERIOD": "100"}, log_sink=None, timeout=120)
    with pytest.raises(LaunchError) as e:
        d.run(_hang_fn)
    assert "heartbeat" in str(e.value)


def _dp_train(steps, batch, seed, use_dp):
    import torch
    import torch.distributed as dist
    from sparkmi.models.mlp import MultilayerPerceptron
    from sparkmi.optim import SGD
    from sparkmi.parallel import DataParallel, init_distributed, world_size, rank
    init_distributed()
    torch.manual_seed(seed)
    model = MultilayerPerceptron([4, 5, 4, 3])
    from sparkmi.utils.flat import FlatParams
    flat = FlatParams(model)
    opt = SGD(flat, lr=0.5)
    ddp = DataParallel(flat) if use_dp else None
    if ddp is not None:
        opt.grad_scale = ddp.grad_scale
    g = torch.Generator().manual_seed(123)
    X = torch.randn(steps * batch * 2, 4, generator=g)
    y = torch.randint(0, 3, (steps * batch * 2,), generator=g)
    ws, r = world_size(), rank()
    per = batch * 2 // ws
    grads_equal = True
    for s in range(steps):
        sl = slice(s * batch * 2 + r * per, s * batch * 2 + (r + 1) * per)
        opt.zero_grad_after_step = False
        loss = model.loss(X[sl], y[sl])
        loss.backward()
        if ddp is not None:
            ddp.finish()
            # Q1 regression: after sync the gradient is identical on every rank
            t = flat.grad.clone()
            dist.broadcast(t, 0)
            grads_equal &= bool(torch.equal(t, flat.grad))
        opt.step()
        flat.zero_grad()
    return flat.master.clone(), grads_equal


def test_data_parallel_parity_and_grad_sync():
    dp_params, eq = Distributor(num_processes=2, use_gpu=False, log_sink=None).run(_dp_train, 5, 8, 0, True)
    assert eq
    single, _ = _dp_train(5, 8, 0, False)
    torch.testing.assert_close(dp_params, single, atol=1e-6, rtol=1e-5)


def test_bucketing_covers_flat_buffer():
    from sparkmi.models.transformer import Transformer
    from sparkmi.parallel import DataParallel
    from sparkmi.utils.flat import FlatParams
    m = Transformer(d_model=64, ffn_hidden=128, num_heads=1, num_layers=2, max_sequence_length=8,
                    src_vocab_size=50, tgt_vocab_size=60)
    flat = FlatParams(m)
    ddp = DataParallel(flat, bucket_mb=0.05)
    spans = [(s, e) for s, e, _ in ddp.buckets]
    assert spans[0][0] == 0 and spans[-1][1] == flat.numel
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert sorted(i for _, _, idx in ddp.buckets for i in idx) == list(range(len(flat.params)))


def test_align_buckets_to_backward_segments():
    """Buckets re-cut at the split-backward segment boundaries: no bucket mixes parameters of
    two segments, the buckets still tile the flat buffer, and complete_buckets() returns exactly
    the buckets of one segment (the StepRunner split path launches those between graphs)."""
    from sparkmi.models.transformer import Transformer
    from sparkmi.parallel import DataParallel
    from sparkmi.utils.flat import FlatParams
    m = Transformer(d_model=64, ffn_hidden=128, num_heads=4, num_layers=2, max_sequence_length=16,
                    src_vocab_size=50, tgt_vocab_size=60)
    flat = FlatParams(m)
    ddp = DataParallel(flat, bucket_mb=0.05)
    top = {id(p) for n, p in m.named_parameters() if n.startswith(("decoder.", "linear."))}
    mid = {id(p) for n, p in m.named_parameters() if n.startswith("encoder.layers.1.")}
    ddp.align_buckets([top, mid])
    seg = lambda p: 0 if id(p) in top else (1 if id(p) in mid else 2)  # noqa: E731
    pos = 0
    for s, e, idx in ddp.buckets:
        assert s == pos and e > s
        pos = e
        assert len({seg(flat.params[i]) for i in idx}) == 1
    assert pos == flat.numel
    w0, w1 = ddp.complete_buckets(top), ddp.complete_buckets(mid)
    assert w0 and w1 and not set(w0) & set(w1)
    assert {i for b in w0 for i in ddp.buckets[b][2]} == {i for i, p in enumerate(flat.params) if id(p) in top}


def _cluster_env():
    import os
    return {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "NODE_RANK",
                                           "GROUP_RANK", "MASTER_ADDR", "SPARKMI_TASK_ADDRS", "SPARKMI_CLUSTER")}


def test_cluster_mode_barrier_tasks():
    """local_mode=False (distributed_cnn.py:227-231): each executor is a barrier task with its own
    node rank and LOCAL_RANK 0; addresses are all-gathered before the run, task 0's is MASTER_ADDR."""
    env = Distributor(num_processes=3, local_mode=False, use_gpu=False, log_sink=None).run(_cluster_env)
    assert env["SPARKMI_CLUSTER"] == "1" and env["RANK"] == "0" and env["WORLD_SIZE"] == "3"
    assert env["LOCAL_RANK"] == "0" and env["LOCAL_WORLD_SIZE"] == "1" and env["NODE_RANK"] == "0"
    addrs = env["SPARKMI_TASK_ADDRS"].split(",")
    assert len(addrs) == 3 and env["MASTER_ADDR"] == addrs[0]


def _cluster_dp():
    import torch
    import torch.distributed as dist
    from sparkmi.parallel import init_distributed
    rank, world, _ = init_distributed()
    t = torch.full((4,), float(rank + 1))
    dist.all_reduce(t)
    return t.tolist(), world


def test_cluster_mode_collectives():
    vals, world = Distributor(num_processes=2, local_mode=False, use_gpu=False, log_sink=None).run(_cluster_dp)
    assert world == 2 and vals == [3.0] * 4


def _collective_hang():
    import time
    import torch
    import torch.distributed as dist
    from sparkmi.parallel import init_distributed
    from sparkmi.runtime import progress
    rank, world, _ = init_distributed(timeout_s=3600)
    for step in range(1, 1000):
        progress(step)
        if rank == 1 and step == 3:
            while True:  # rank 1 wedges: rank 0 blocks INSIDE all_reduce, its heartbeat thread still beats
                time.sleep(1)
        dist.all_reduce(torch.ones(4))
        time.sleep(0.05)


def test_hang_inside_collective_detected_by_progress():
    d = Distributor(num_processes=2, use_gpu=False, progress_timeout=3.0, log_sink=None, timeout=120)
    with pytest.raises(LaunchError) as e:
        d.run(_collective_hang)
    assert "progress stalled" in str(e.value)
