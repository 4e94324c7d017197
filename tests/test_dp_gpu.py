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
    ddp = DataParallel(flat, bucket_mb=0.5, ipc=False)  # the process-group path (RCCL on a multi-GPU node)
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


# ---- transformer DP parity grid (the GPU kernel path): 2 ranks x batch 4 == 1 rank x batch 8 ----
_CFGS = [  # name, optimizer, zero, graph, split, ipc
    ("sgd_eager", "sgd", False, False, False, False),
    ("sgd_graph", "sgd", False, True, False, False),
    ("sgd_split", "sgd", False, True, True, False),
    ("sgd_ipc_eager", "sgd", False, False, False, True),
    ("sgd_ipc_graph", "sgd", False, True, False, True),
    ("adam_eager", "adam", False, False, False, False),
    ("adam_zero_eager", "adam", True, False, False, False),
    ("adam_graph", "adam", False, True, False, False),
    ("adam_zero_graph", "adam", True, True, False, False),
    ("adam_split", "adam", False, True, True, False),
    ("adam_zero_split", "adam", True, True, True, False),
    # the IPC kernels on their comm stream under the split-graph backward (buckets reduced while
    # the next backward piece replays), two-shot forced (2 ranks would pick one-shot)
    ("sgd_ipc2_eager", "sgd", False, False, False, 2),
    ("sgd_ipc2_split", "sgd", False, True, True, 2),
    ("adam_ipc2_split", "adam", False, True, True, 2),
    ("adam_ipc2_graph", "adam", False, True, False, 2),
    # the zero-copy IPC two-shot (3): peers read each other's registered flat gradient in place
    ("sgd_zc_split", "sgd", False, True, True, 3),
    ("adam_zc_graph", "adam", False, True, False, 3),
    ("adam_zc_eager", "adam", False, False, False, 3),
    # "_1u": one optimizer update after every bucket (PER_BUCKET_OPT off) — the per-bucket update
    # (each bucket's Adam behind its own RCCL work / IPC event) must equal it bit for bit
    ("adam_eager_1u", "adam", False, False, False, False),
    ("adam_zero_split_1u", "adam", True, True, True, False),
    ("adam_split_1u", "adam", False, True, True, False),
    ("adam_ipc2_split_1u", "adam", False, True, True, 2),
    ("adam_ipc2_graph_1u", "adam", False, True, False, 2),
]


def _dp_grid(steps, only=None):
    import torch
    from sparkmi.models.transformer import Transformer
    from sparkmi.ops.rng import reset_salts
    from sparkmi.optim import SGD, Adam
    from sparkmi.parallel import DataParallel, init_distributed
    from sparkmi.parallel import ddp as ddp_mod
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    rank, world, device = init_distributed()
    g = torch.Generator().manual_seed(1)
    data = torch.randint(4, 300, (steps, 2, 8, 64), generator=g).to(device)  # no padding: equal token counts
    per = 8 // world
    out = {}
    for name, ok, zero, graph, split, ipc in _CFGS:
        if world == 1 and name not in ("sgd_eager", "adam_eager"):
            continue
        if only is not None and name not in only:
            continue
        ddp_mod.PER_BUCKET_OPT = not name.endswith("_1u")
        reset_salts()
        torch.manual_seed(0)
        m = Transformer(d_model=128, ffn_hidden=256, num_heads=2, drop_prob=0.0, num_layers=2, max_sequence_length=64,
                        src_vocab_size=300, tgt_vocab_size=300, emb_dropout=0.0, dtype="fp32").to(device)
        flat = FlatParams(m, shadow=False)
        opt = SGD(flat, lr=0.05) if ok == "sgd" else Adam(flat, lr=1e-3)
        ddp = (DataParallel(flat, bucket_mb=0.5, zero=zero, ipc=bool(ipc), comm="ipc_zc" if ipc == 3 else None)
               if world > 1 else None)
        if ddp is not None:
            assert (ddp.ipc is not None) == bool(ipc), name
            assert (ddp.comm == "ipc_zc") == (ipc == 3), name
            if ipc == 2:
                ddp.ipc.force_algo = 2
        split_fn = (lambda mm, s, t: mm.training_step_split(s, t)) if split else None
        runner = StepRunner(m, lambda mm, s, t: mm.training_step_loss(s, t), opt, ddp, graph=graph, warmup_eager=2,
                            split_fn=split_fn)
        if ddp is not None:
            assert (ddp._bopt is not None) == (ok == "adam" and ddp_mod.PER_BUCKET_OPT), name
        for i in range(steps):
            runner.step(data[i, 0, rank * per:(rank + 1) * per].contiguous(),
                        data[i, 1, rank * per:(rank + 1) * per].contiguous())
        torch.cuda.synchronize()
        out[name] = flat.master.cpu().clone()
        if ddp is not None:
            ddp.check()
            ddp.close()
        del runner, opt, ddp, flat, m
    ddp_mod.PER_BUCKET_OPT = True
    import torch.distributed as dist
    if world == 1:
        return [out]
    allr = [None] * world
    dist.all_gather_object(allr, out)  # launch() returns rank 0's value: hand it every rank's
    return allr


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_transformer_dp_parity_grid():
    """fp32 transformer on the GPU kernels (split-plane GEMMs, fused attention / LN): two ranks
    sharing the GPU with batch 4 each == one rank with batch 8 — eager, whole-step HIP graph and
    split-graph (overlapped bucket reduction) steps, over the process group (gloo here, RCCL on a
    node) and over the xGMI IPC kernel; and with Adam, ZeRO-1 (reduce-scatter, sharded update,
    all-gather) is BITWISE equal to the replicated update for every step mode (2-operand sums
    commute exactly)."""
    env = {"SPARKMI_DIST_BACKEND": "gloo"}
    r2 = launch(_dp_grid, (5,), {}, num_processes=2, use_gpu=True, env=env, log_sink=None, timeout=380)
    (r1,) = launch(_dp_grid, (5,), {}, num_processes=1, use_gpu=True, env=env, log_sink=None, timeout=380)
    a, b = r2
    for name in a:
        assert torch.equal(a[name], b[name]), f"{name}: ranks disagree"
    for name in ("sgd_eager", "sgd_graph", "sgd_split", "sgd_ipc_eager", "sgd_ipc_graph"):
        torch.testing.assert_close(a[name], r1["sgd_eager"], rtol=1e-4, atol=1e-5, msg=name)
    # Adam: sign-like updates amplify last-bit gradient differences on ~zero gradients, so the
    # 2 x 4 vs 1 x 8 comparison is loose; ZeRO on / off must agree exactly
    assert (a["adam_eager"] - r1["adam_eager"]).abs().max() < 5 * 1e-3 * 5
    for mode in ("eager", "graph", "split"):
        assert torch.equal(a[f"adam_zero_{mode}"], a[f"adam_{mode}"]), mode
    # IPC two-shot on the comm stream: the split-graph step equals the eager step bit for bit
    # (same rank-order sums), and both agree with the process-group path to fp32 tolerance
    assert torch.equal(a["sgd_ipc2_split"], a["sgd_ipc2_eager"])
    torch.testing.assert_close(a["sgd_ipc2_eager"], r1["sgd_eager"], rtol=1e-4, atol=1e-5)
    assert (a["adam_ipc2_split"] - r1["adam_eager"]).abs().max() < 5 * 1e-3 * 5
    assert torch.equal(a["adam_ipc2_graph"], a["adam_ipc2_split"])
    # zero-copy two-shot: the staged two-shot's rank-order sums, bit for bit
    assert torch.equal(a["sgd_zc_split"], a["sgd_ipc2_split"])
    assert torch.equal(a["adam_zc_graph"], a["adam_ipc2_graph"])
    assert torch.equal(a["adam_zc_eager"], a["adam_ipc2_graph"])
    # the optimizer per bucket == one update after every bucket, bit for bit
    for name in ("adam_eager", "adam_zero_split", "adam_split", "adam_ipc2_split", "adam_ipc2_graph"):
        assert torch.equal(a[name], a[name + "_1u"]), name


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_transformer_dp_parity_grid_world4():
    """The same grid at FOUR ranks sharing the GPU (batch 2 each == one rank at batch 8): the
    4-chunk two-shot ranges, the 4-way ZeRO-1 pieces and the IPC split-graph path, which the
    2-rank grid cannot reach."""
    env = {"SPARKMI_DIST_BACKEND": "gloo"}
    only = ("sgd_eager", "sgd_split", "sgd_ipc_eager", "sgd_ipc2_split", "adam_eager", "adam_zero_eager",
            "adam_zero_split", "adam_split", "adam_zero_split_1u", "adam_split_1u", "sgd_zc_split", "adam_zc_graph")
    r4 = launch(_dp_grid, (4, only), {}, num_processes=4, use_gpu=True, env=env, log_sink=None, timeout=380)
    (r1,) = launch(_dp_grid, (4,), {}, num_processes=1, use_gpu=True, env=env, log_sink=None, timeout=380)
    for name in r4[0]:
        for q in r4[1:]:
            assert torch.equal(r4[0][name], q[name]), f"{name}: ranks disagree"
    a = r4[0]
    for name in ("sgd_eager", "sgd_split", "sgd_ipc_eager", "sgd_ipc2_split"):
        torch.testing.assert_close(a[name], r1["sgd_eager"], rtol=1e-4, atol=1e-5, msg=name)
    # 4-operand sums: the reduce-scatter and the all-reduce may associate differently, and Adam's
    # sign-like first steps amplify last-bit differences on ~zero gradients (bound as above)
    assert (a["adam_zero_eager"] - a["adam_eager"]).abs().max() < 5 * 1e-3 * 4
    assert (a["adam_zero_split"] - a["adam_split"]).abs().max() < 5 * 1e-3 * 4
    assert (a["adam_eager"] - r1["adam_eager"]).abs().max() < 5 * 1e-3 * 4
    for name in ("adam_zero_split", "adam_split"):
        assert torch.equal(a[name], a[name + "_1u"]), name
    # zero-copy two-shot at 4 ranks (4-chunk ranges): the staged kernel's sums, bit for bit
    assert torch.equal(a["sgd_zc_split"], a["sgd_ipc2_split"])
    assert (a["adam_zc_graph"] - r1["adam_eager"]).abs().max() < 5 * 1e-3 * 4


# ---- small models over the IPC kernels: the whole-step graph and the two-shot path ----
def _small_dp(kind, steps, graph, sparse=False):
    import torch
    from sparkmi.models.lstm import LSTM
    from sparkmi.models.mlp import MultilayerPerceptron
    from sparkmi.optim import SGD
    from sparkmi.parallel import DataParallel, init_distributed
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    rank, world, device = init_distributed()
    torch.manual_seed(0)
    g = torch.Generator().manual_seed(5)
    GB = 8  # global batch
    if kind == "mlp":
        m = MultilayerPerceptron((4, 5, 4, 3)).to(device)
        xs = torch.randn(steps, GB, 4, generator=g).to(device)
        ys = torch.randint(0, 3, (steps, GB), generator=g).to(device)
        loss_fn = lambda mm, x, y: mm.loss(x, y)  # noqa: E731
    else:
        # 5000 x 32 embedding: a 640 KB gradient bucket (two-shot at 4 ranks, auto-selected)
        m = LSTM(5000, 32, 32, 4, num_layers=2, dropout=0.0).to(device)
        xs = torch.randint(4, 5000, (steps, GB, 24), generator=g).to(device)
        ys = torch.randint(0, 4, (steps, GB), generator=g).to(device)
        loss_fn = lambda mm, x, y: mm.loss(x, y)[0]  # noqa: E731
    flat = FlatParams(m, shadow=False)
    opt = SGD(flat, lr=0.1)
    ddp = DataParallel(flat, bucket_mb=64.0, sparse_rows=m.sparse_rows() if sparse else None) if world > 1 else None
    info = None
    if ddp is not None and not sparse:
        assert ddp.ipc is not None, "small gradients take the IPC kernels in auto mode"
        n = max(e - s for s, e, _ in ddp.buckets)
        info = ddp.ipc.algo_for(n)
    runner = StepRunner(m, loss_fn, opt, ddp, graph=graph, warmup_eager=2)
    per = GB // world
    for i in range(steps):
        runner.step(xs[i, rank * per:(rank + 1) * per].contiguous(), ys[i, rank * per:(rank + 1) * per].contiguous())
    torch.cuda.synchronize()
    if ddp is not None:
        ddp.check()
        ddp.close()
    return flat.master.cpu().clone(), info


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_mlp_ipc_whole_step_graph_matches_single_process():
    """MLP data parallelism with the WHOLE step (forward, backward, IPC all-reduce, SGD) as one
    HIP graph == one process at twice the batch (restored from round 2)."""
    env = {"SPARKMI_DIST_BACKEND": "gloo"}
    p2, algo = launch(_small_dp, ("mlp", 8, True), {}, num_processes=2, use_gpu=True, env=env, log_sink=None,
                      timeout=280)
    p1, _ = launch(_small_dp, ("mlp", 8, False), {}, num_processes=1, use_gpu=True, env=env, log_sink=None, timeout=280)
    assert algo == 1
    torch.testing.assert_close(p2, p1, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_lstm_dp_auto_two_shot_matches_single_process():
    """A 640 KB LSTM gradient at 4 ranks: auto mode picks the IPC TWO-shot kernel; 4 ranks x batch
    2 == one process x batch 8 (graph-captured steps)."""
    env = {"SPARKMI_DIST_BACKEND": "gloo"}
    p4, algo = launch(_small_dp, ("lstm", 5, True), {}, num_processes=4, use_gpu=True, env=env, log_sink=None,
                      timeout=380)
    p1, _ = launch(_small_dp, ("lstm", 5, False), {}, num_processes=1, use_gpu=True, env=env, log_sink=None,
                   timeout=380)
    assert algo == 2
    torch.testing.assert_close(p4, p1, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_lstm_dp_sparse_embedding_matches_single_process():
    """The row-sparse embedding-gradient exchange on device tensors (sort / dedup / rank-order
    scatter-add on the GPU; the dense rest over IPC): 2 ranks x batch 4 == one process x batch 8,
    forward + backward graph-captured."""
    env = {"SPARKMI_DIST_BACKEND": "gloo"}
    p2, _ = launch(_small_dp, ("lstm", 5, True, True), {}, num_processes=2, use_gpu=True, env=env, log_sink=None,
                   timeout=280)
    p1, _ = launch(_small_dp, ("lstm", 5, False), {}, num_processes=1, use_gpu=True, env=env, log_sink=None,
                   timeout=280)
    torch.testing.assert_close(p2, p1, rtol=1e-4, atol=1e-5)


# ---- the data-parallel CNN fast step: fused gradient kernel + IPC + SGD ----
def _cnn_dp(steps, graph, bind, dtype="fp32", fuse_sgd=True):
    import torch
    from sparkmi.data.synthetic import fashion_mnist_like
    from sparkmi.models.cnn import FashionMNISTModel
    from sparkmi.optim import SGD
    from sparkmi.parallel import DataParallel, init_distributed
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    rank, world, device = init_distributed()
    torch.manual_seed(0)
    m = FashionMNISTModel(1, 10, 10, dtype=dtype).to(device)
    flat = FlatParams(m, shadow=False)
    opt = SGD(flat, lr=0.05)
    from sparkmi.parallel import ddp as D
    D.FUSE_SGD = fuse_sgd
    ddp = DataParallel(flat) if world > 1 else None
    GB = 32
    imgs, labels = fashion_mnist_like(steps * GB, seed=3, device=device)
    per = GB // world
    batches = [(imgs[i * GB + rank * per:i * GB + (rank + 1) * per].contiguous(),
                labels[i * GB + rank * per:i * GB + (rank + 1) * per].contiguous()) for i in range(steps)]
    runner = StepRunner(m, lambda mm, x, y: mm.loss(x, y), opt, ddp, graph=graph, warmup_eager=2,
                        fused_step=(lambda mm, o, x, y: mm.fused_sgd_step(o, x, y)) if world == 1 else None,
                        fused_grad=(lambda mm, x, y: mm.fused_grad_step(x, y)) if world > 1 else None,
                        bind_inputs=bind)
    if bind:
        runner.unroll = 2
        runner.run_steps(batches[:3])
        runner.run_steps(batches[3:])
    else:
        for b in batches:
            runner.step(*b)
    torch.cuda.synchronize()
    comm = None
    if ddp is not None:
        comm = (ddp.comm, ddp.last_step_fused, float(opt.step_t.item()))
        ddp.check()
        ddp.close()
    import torch.distributed as dist
    out = flat.master.cpu().clone()
    if world == 1:
        return [out], comm
    allr = [None] * world
    dist.all_gather_object(allr, out)
    return allr, comm


@pytest.mark.gpu
@pytest.mark.timeout(400)
@pytest.mark.parametrize("world", [2, 4])
def test_cnn_dp_fused_step_matches_single_process(world):
    """FashionMNISTModel data parallelism on the fast step: the fused kernel's gradient mode (batch
    gradient added to the flat buffer in its ticketed tail), the IPC one-shot all-reduce and SGD,
    eager and in bound multi-step HIP graphs.  Parameters are bitwise equal on every rank, and
    world x (32 / world) == one process x 32 (the fused SGD step) to fp32 tolerance (different
    summation orders)."""
    env = {"SPARKMI_DIST_BACKEND": "gloo"}
    (r1,), _ = launch(_cnn_dp, (7, False, False), {}, num_processes=1, use_gpu=True, env=env, log_sink=None,
                      timeout=300)
    for graph, bind in ((False, False), (True, True)):
        rs, comm = launch(_cnn_dp, (7, graph, bind), {}, num_processes=world, use_gpu=True, env=env, log_sink=None,
                          timeout=300)
        assert comm[0] == "ipc" and comm[1], comm  # the SGD step ran inside the reduction (ddp.fuse_sgd)
        assert comm[2] == 7.0, comm                 # and advanced the step counter once per step
        for q in rs[1:]:
            assert torch.equal(rs[0], q), "ranks disagree"
        torch.testing.assert_close(rs[0], r1, rtol=1e-4, atol=2e-6, msg=f"graph={graph} bind={bind}")
        # the reduction's SGD epilogue is bitwise the separate SGD launch
        rs2, comm2 = launch(_cnn_dp, (7, graph, bind, "fp32", False), {}, num_processes=world, use_gpu=True, env=env,
                            log_sink=None, timeout=300)
        assert not comm2[1] and comm2[2] == 7.0, comm2
        assert torch.equal(rs2[0], rs[0]), f"fused SGD != sgd_kernel (graph={graph} bind={bind})"


# ---- the bulk-gradient probe with its four candidates on the GPU ----
def _probe_gpu():
    import torch
    from sparkmi.parallel import ddp, init_distributed
    from sparkmi.utils.flat import FlatParams
    rank, world, dev = init_distributed()
    ddp.IPC_LIMIT_BYTES = 1024  # a "bulk" gradient at test size: the start-up probe runs
    torch.manual_seed(0)
    flat = FlatParams(torch.nn.Sequential(torch.nn.Linear(512, 512), torch.nn.Linear(512, 512)).to(dev),
                      shadow=False)
    dp = ddp.DataParallel(flat, bucket_mb=0.5)
    out = dict(dp.comm_probe)
    out["comm"] = dp.comm
    ok = True
    for it in range(3):  # the chosen path reduces every bucket exactly (two operands commute)
        flat.grad.fill_(float(rank + 1 + it))
        dp.finish()
        torch.cuda.synchronize()
        ok = ok and bool((flat.grad == float(sum(r + 1 + it for r in range(world)))).all())
    dp.check()
    dp.close()
    out["ok"] = ok
    return out


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_dp_probe_measures_zero_copy_candidate(world):
    """Ranks sharing the GPU: the start-up probe registers every rank's flat gradient, measures the
    staged AND the zero-copy IPC two-shot (both pass their exact-sum checks) and the process group,
    and the path it keeps reduces exactly."""
    res = launch(_probe_gpu, (), {}, num_processes=world, use_gpu=True, env={"SPARKMI_DIST_BACKEND": "gloo"},
                 log_sink=None, timeout=280)
    assert res["ipc_ms"] is not None and res["ipc_zc_ms"] is not None and res["rccl_ms"] is not None, res
    assert res["choice"] == res["comm"] and res["ok"], res
