#!/usr/bin/env python3
"""Headline benchmark: whole-node training samples/sec of the reference workloads on MI355X.

Flagship = the BASELINE.json transformer config: encoder-decoder Transformer (transformer.py),
6 layers, d_model 512, 8 heads, ffn 1024, seq 256, vocab 10k/10k, batch 32 per GPU, Adam
lr 1e-3, dropout 0.1, reference mask semantics — a full training step (forward, masked token
CE, backward, gradient all-reduce, optimizer) per iteration, synthetic Multi30k-shaped data
resident in HBM, random-init weights.  ``value`` is measured at the REFERENCE precision: fp32
activations, fp32 weights, fp32 accumulation, exactly as the reference trains
(pytorch_machine_translator.py:120-137, default fp32 modules).  GEMM products are exact: every fp32
operand is carried as three bf16 planes (hi + mid + lo, split once where it is produced) and the
six significant plane products run on the bf16 matrix cores (csrc/kernels/gemm_sp*.hip; measured
error against fp64 at or below the v_mfma_f32_32x32x2_f32 kernel, tests/test_gemm_sp_gpu.py; the
same step on that f32-MFMA kernel is reported beside it as ``transformer_fp32_f32mfma``).  Every
model is built after resetting the dropout salt sequence and the torch seed, so its trajectory
does not depend on which models ran before it in the process; the headline run's per-step losses
are in ``losses``.  The bf16
(fp32-master) variant of the same step and the distributed_cnn workload (the other half of the
BASELINE metric) are reported beside it for the same N, plus the LSTM / MLP workloads.

Contract: ``python bench.py --gpus N --steps K --warmup W``.  Multi-GPU runs are launched by
torch.distributed.run (one rank per GPU, RCCL); when ``--gpus N > 1`` is given WITHOUT a
launcher (no WORLD_SIZE in the environment) this script spawns the N ranks itself before any
GPU call (reference launch: distributed_cnn.py:227-231, TorchDistributor(num_processes=N)).
W untimed warm-up steps, then K steps timed between barrier+synchronize on both sides; the MAX
elapsed over ranks is used; rank 0 prints one JSON line.  ``value`` = whole-job samples/s =
N * batch * K / max_elapsed (weak scaling).
"""
import argparse
import math
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# transformer L6/S256/B32 CPU proxy, best whole-node figure (1 proc x 8 threads)
BASELINE_TRANSFORMER = 4.79
BASELINE_CNN = 5655.0
BASELINE_LSTM = 1365.0    # 1 proc x 8 threads
BASELINE_MLP = 130476.0   # world 1, 1 thread
METRIC = "samples/sec (whole node) distributed_cnn + transformer at 1/2/4/8 MI355X"
F32_PRECISION = ("fp32 activations/weights/gradients/accumulators (reference precision); GEMM products exact: "
                 "fp32 operands carried as 3 bf16 planes (hi+mid+lo, split once where produced), 6 plane products "
                 "on v_mfma_f32_16x16x32_bf16 (error vs fp64 at or below the f32-MFMA kernel: "
                 "tests/test_gemm_sp_gpu.py); fp32 attention products on the same exact 3-way bf16 split")
SPLIT_PEAK_TF = 2500.0 / 6  # 6 bf16 products per fp32 product on the 2.5 PF (spec) bf16 matrix cores
# measured on this MI355X (profiles/r3_bf16_peak_rate.log, tools/bench_bf16_peak.py): hipBLASLt bf16
# 8192^3 on random data sustains 1,268 TF — the chip lowers its clock under MFMA load on random
# operands (1,738 TF on zeros) — so the practical ceiling of the 6-product fp32 GEMM is ~211 TF
BF16_MEASURED_TF = 1268.0
SPLIT_MEASURED_TF = BF16_MEASURED_TF / 6


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="all", choices=["all", "transformer", "cnn", "aux"])
    ap.add_argument("--dtype", default="auto", choices=["auto", "fp32", "bf16", "both"],
                    help="transformer compute dtype; auto = fp32 headline + bf16 beside it on GPU, fp32 on CPU")
    ap.add_argument("--device", default="auto", choices=["auto", "cpu", "cuda"])
    ap.add_argument("--aux-steps", type=int, default=100, help="timed steps of the LSTM / MLP extras")
    ap.add_argument("--cnn-batch", type=int, default=32)
    ap.add_argument("--cnn-steps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=256)
    ap.add_argument("--layers", type=int, default=6)
    ap.add_argument("--vocab", type=int, default=10000)
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"])
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--split", type=int, default=1, help="multi-graph backward with overlapped all-reduce (DP)")
    ap.add_argument("--no-aux", action="store_true", help="skip the LSTM / MLP extras")
    ap.add_argument("--data", default="random", choices=["random", "copy"],
                    help="transformer batches: random = independent uniform src/tgt (Multi30k-shaped; loss floor "
                         "ln(V-4)), copy = tgt a fixed permutation of src (learnable, same shapes)")
    ap.add_argument("--no-zero-compare", action="store_true",
                    help="skip the ZeRO-1 variant of the fp32 transformer step (measured only when N > 1)")
    ap.add_argument("--no-f32-compare", action="store_true",
                    help="skip the f32-MFMA comparison run of the fp32 transformer step")
    return ap.parse_args(argv)


def spawn_ranks(n, argv):
    """Launch ``n`` ranks of this script (torchrun env contract, 127.0.0.1 rendezvous) and
    relay rank 0's stdout.  Runs in a process that has not touched the GPU, and never execs."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                    "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                    "PYTHONUNBUFFERED": "1"})
        env.setdefault("OMP_NUM_THREADS", "1")
        out = None if r == 0 else subprocess.DEVNULL
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env, stdout=out))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                c = p.poll()
                if c is None:
                    continue
                procs.remove(p)
                if c != 0:
                    rc = c
                    for q in procs:  # one rank failed: the group cannot finish its collectives
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
    return rc


def _sync(device):
    import torch
    if device.type == "cuda":
        torch.cuda.synchronize()


def fresh_model_state(seed):
    """Reset the process-global dropout salt sequence and the torch seed before building a model:
    its masks and init then do not depend on the models built before it in this process."""
    import torch
    from sparkmi.ops.rng import reset_salts
    reset_salts()
    torch.manual_seed(seed)


def time_steps(runner, batches, steps, warmup, device, world, record=None):
    """``record``: a list that receives each timed step's loss (a device copy, read after timing)."""
    import torch
    from sparkmi.parallel import barrier
    # the HIP-graph capture must happen inside the untimed warm-up: eager steps first, the
    # capture on the last warm-up step (StepRunner captures on step warmup_eager + 1)
    runner.warmup_eager = max(0, min(runner.warmup_eager, warmup - 1))
    n = len(batches)
    bind = getattr(runner, "bind_inputs", False) and record is None
    if bind:
        # HBM-resident batches read in place (no per-step input copy), each cycle over the n
        # batches one multi-step graph (one launch per n steps): every capture happens in the
        # untimed warm-up, which replays the timed sequence once
        warmup = max(warmup, runner.warmup_eager + n + 1)
        runner.unroll = n
    loss = None
    for i in range(warmup):
        loss = runner.step(*batches[i % n])
    seq = [batches[i % n] for i in range(steps)]
    if bind:
        loss = runner.run_steps(seq)
    _sync(device)
    barrier()
    _sync(device)
    t0 = time.perf_counter()
    if bind:
        loss = runner.run_steps(seq)
    for i in range(0 if bind else steps):
        loss = runner.step(*batches[i % n])
        if record is not None:
            record.append(loss.detach().clone())
    _sync(device)
    barrier()
    _sync(device)
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, loss


def ranks_in_sync(flat, world):
    """After the timed steps every rank must hold bit-identical parameters (synchronous data
    parallelism): rank 0's master weights broadcast and compared on every rank (None at N = 1)."""
    if world <= 1:
        return None
    import torch
    import torch.distributed as dist
    ref = flat.master.clone()
    dist.broadcast(ref, 0)
    ok = torch.tensor([1 if torch.equal(ref, flat.master) else 0], dtype=torch.int32, device=ref.device)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    return bool(int(ok.item()))


def time_allreduce(flat, device, world, iters=10):
    """Isolated cost of the step's gradient all-reduce (the whole flat fp32 gradient buffer,
    same buckets and backend as the step): the communication phase, in ms, max over ranks."""
    if world <= 1:
        return None
    import torch
    import torch.distributed as dist
    g = flat.grad
    for _ in range(2):
        dist.all_reduce(g)
    _sync(device)
    from sparkmi.parallel import barrier
    barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(g)
    _sync(device)
    el = (time.perf_counter() - t0) / iters
    t = torch.tensor([el], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return round(float(t.item()) * 1000, 3)


def time_comm_paths(device, world, bucket_mb, iters=5):
    """The bulk-gradient collective options at one bucket (``--bucket-mb``), ms per all-reduce,
    max over ranks: RCCL with its default channels, RCCL on a communicator created with
    min_ctas = 32 (more channels over the 7 xGMI links), and the IPC two-shot kernel
    (csrc/comm/ipc_allreduce.hip).  DataParallel's start-up probe makes the same IPC-vs-RCCL
    choice for the run (``comm_probe`` of the step result)."""
    if world <= 1 or device.type != "cuda":
        return None
    import torch
    import torch.distributed as dist
    n = int(bucket_mb * (1 << 20) / 4) // 4 * 4
    x = torch.zeros(n, dtype=torch.float32, device=device)

    def timed(fn):
        for _ in range(2):
            fn()
        _sync(device)
        dist.all_reduce(torch.zeros(1, device=device))
        _sync(device)
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        _sync(device)
        t = torch.tensor([(time.perf_counter() - t0) / iters * 1e3], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return round(float(t.item()), 3)

    out = {"bucket_bytes": n * 4}
    out["rccl_ms"] = timed(lambda: dist.all_reduce(x))
    if dist.get_backend() == "nccl":
        try:
            opts = dist.ProcessGroupNCCL.Options()
            opts.config.min_ctas = 32
            g = dist.new_group(list(range(world)), backend="nccl", pg_options=opts)
            out["rccl_min_ctas32_ms"] = timed(lambda: dist.all_reduce(x, group=g))
            dist.destroy_process_group(g)
        except Exception as e:  # noqa: BLE001 — reported, not fatal
            out["rccl_min_ctas32_ms"] = f"unavailable: {type(e).__name__}"
    try:
        from sparkmi.parallel.comm import IpcAllReduce
        ar = IpcAllReduce(cap_floats=n)
        out["ipc_two_shot_ms"] = timed(lambda: ar(x, algo=2))
        ar.check()
        ar.close()
    except Exception as e:  # noqa: BLE001
        out["ipc_two_shot_ms"] = f"unavailable: {type(e).__name__}"
    for k in ("rccl_ms", "rccl_min_ctas32_ms", "ipc_two_shot_ms"):
        v = out.get(k)
        if isinstance(v, float) and v > 0:
            out[k.replace("_ms", "_GBps_busbw")] = round(2 * (world - 1) / world * n * 4 / (v * 1e-3) / 1e9, 1)
    return out


def bench_cnn(args, rank, world, device, dtype="fp32"):
    """distributed_cnn.py workload: FashionMNISTModel, batch 32/GPU, SGD lr 0.01, mean CE."""
    import torch
    from sparkmi.data.synthetic import fashion_mnist_like
    from sparkmi.models.cnn import FashionMNISTModel
    from sparkmi.optim import SGD
    from sparkmi.parallel.ddp import DataParallel
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    fresh_model_state(4321)
    model = FashionMNISTModel(1, 10, 10, dtype=dtype).to(device).train()
    flat = FlatParams(model)
    opt = SGD(flat, lr=0.01)
    ddp = DataParallel(flat) if world > 1 else None
    use_graph = device.type == "cuda" and args.graph != "off"
    # one executor: the whole step (forward, backward, batch gradient sum, SGD) is ONE launch;
    # data-parallel: the same kernel leaves the batch gradient (gradient mode), then the IPC
    # all-reduce and SGD — three launches, in bound multi-step graphs like the single-executor step
    fused = (lambda m, o, x, y: m.fused_sgd_step(o, x, y)) if world == 1 else None
    fgrad = (lambda m, x, y: m.fused_grad_step(x, y)) if world > 1 else None
    runner = StepRunner(model, lambda m, x, y: m.loss(x, y), opt, ddp, graph=use_graph, fused_step=fused,
                        bind_inputs=True, fused_grad=fgrad)
    imgs, labels = fashion_mnist_like(16 * args.cnn_batch, seed=7 + rank, device=device)
    batches = [(imgs[i * args.cnn_batch:(i + 1) * args.cnn_batch], labels[i * args.cnn_batch:(i + 1) * args.cnn_batch])
               for i in range(16)]
    elapsed, loss = time_steps(runner, batches, args.cnn_steps, max(args.warmup, 5), device, world)
    ar = time_allreduce(flat, device, world)
    comm = None
    if ddp is not None:
        comm = ddp.comm
        ddp.close()
    v = world * args.cnn_batch * args.cnn_steps / elapsed
    return {"samples_per_s": round(v, 1), "ms_per_step": round(elapsed / args.cnn_steps * 1000, 4),
            "vs_baseline": round(v / BASELINE_CNN, 2), "final_loss": round(float(loss), 4),
            "dtype": dtype, "global_batch": world * args.cnn_batch, "steps": args.cnn_steps,
            "allreduce_ms": ar, "grad_bytes": flat.numel * 4, "comm": comm,
            "config": f"FashionMNISTModel fused HIP kernel ({'bf16 MFMA' if dtype == 'bf16' else 'fp32'} convs), "
                      f"batch {args.cnn_batch}/GPU, SGD lr0.01, dp{world}",
            "baseline_ref": "BASELINE.md §2 CNN CPU proxy 5,655 samples/s (1 proc x 8 threads)"}


def bench_cnn_recipe(args, rank, world, device, dtype="bf16"):
    """The CNN exactly as the recipe trains it (sparkmi/recipes/cnn.py -> Trainer.fit): a 60,000-image
    HBM-resident uint8 shard per executor, a fresh shuffle every epoch, each step gathering its batch
    inside the step graph (DeviceLoader fixed=True), multi-step graphs of ``unroll`` steps, device-side
    loss metrics — the path a user of examples/distributed_cnn.py gets, timed like the headline CNN
    step (both numbers side by side)."""
    import dataclasses
    import torch
    from sparkmi.data.dataset import DeviceLoader
    from sparkmi.data.synthetic import fashion_mnist_like
    from sparkmi.models.cnn import FashionMNISTModel
    from sparkmi.optim import SGD
    from sparkmi.parallel import barrier
    from sparkmi.recipes.cnn import CNNConfig
    from sparkmi.train.trainer import Trainer
    fresh_model_state(4321)
    n = 60000
    x, y = fashion_mnist_like(n, seed=17 + rank)
    cfg = CNNConfig(world=world, batch_size=args.cnn_batch, lr=0.01, conv_dtype=dtype, log_every=10 ** 9,
                    verbose=False, graph=args.graph != "off")
    loader = DeviceLoader([x, y], cfg.batch_size, device, shuffle=True, drop_last=True, seed=1000 * rank, fixed=True)
    model = FashionMNISTModel(1, 10, 10, dtype=dtype)
    tr = Trainer(model, lambda m, a, b: m.loss(a, b), lambda flat: SGD(flat, lr=cfg.lr), cfg, device, rank, world,
                 "cnn_bench", shadow=False, fused_step=lambda m, o, a, b: m.fused_sgd_step(o, a, b),
                 fused_grad=lambda m, a, b: m.fused_grad_step(a, b))
    warm = max(args.warmup, 5) + 2 * tr.runner.unroll
    tr.cfg = dataclasses.replace(cfg, max_steps=warm)
    tr.fit(loader, 10 ** 6)
    _sync(device)
    barrier()
    _sync(device)
    t0 = time.perf_counter()
    # one whole epoch of the shard (or more): the per-fit setup (epoch shuffle, loader reset) is
    # amortised as in a real run instead of dominating a short timed window
    timed = max(args.cnn_steps, n // cfg.batch_size)
    tr.cfg = dataclasses.replace(cfg, max_steps=warm + timed)
    res = tr.fit(loader, 10 ** 6)
    _sync(device)
    barrier()
    _sync(device)
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    steps = res["steps"]
    gather = "in the step kernel" if tr.runner.pre_step is None else "in the step graph"
    tr.close()
    v = world * args.cnn_batch * steps / elapsed
    return {"samples_per_s": round(v, 1), "ms_per_step": round(elapsed / steps * 1000, 4), "steps": steps,
            "final_loss": round(res["final_loss"], 4), "dtype": dtype, "global_batch": world * args.cnn_batch,
            "vs_baseline": round(v / BASELINE_CNN, 2),
            "config": f"Trainer.fit over a shuffled 60k-image HBM shard per executor, batch gather {gather}, "
                      f"{cfg.unroll}-step graphs, dp{world}"}


def bench_lstm(args, rank, world, device):
    """distributed_lstm.py workload: Embedding(V~95.8k, 32) -> LSTM(32, 32, 2 layers, dropout 0.5)
    -> fc(4) at every step, CE on the last step; batch 32/GPU, T = 129, Adam lr 1e-3."""
    import torch
    from sparkmi.models.lstm import LSTM
    from sparkmi.optim import Adam
    from sparkmi.parallel.ddp import DataParallel
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    V, B, T = 95812, 32, 129
    fresh_model_state(11)
    model = LSTM(V, 32, 32, 4, num_layers=2, padding_idx=7).to(device).train()
    flat = FlatParams(model, shadow=False)
    opt = Adam(flat, lr=1e-3)
    ddp = DataParallel(flat) if world > 1 else None
    runner = StepRunner(model, lambda m, x, y: m.loss(x, y)[0], opt, ddp, graph=device.type == "cuda" and args.graph != "off",
                        bind_inputs=True)
    g = torch.Generator().manual_seed(21 + rank)
    batches = [(torch.randint(0, V, (B, T), generator=g).to(device), torch.randint(0, 4, (B,), generator=g).to(device))
               for _ in range(8)]
    steps = args.aux_steps
    elapsed, _ = time_steps(runner, batches, steps, max(args.warmup, 5), device, world)
    if ddp is not None:
        ddp.close()
    v = world * B * steps / elapsed
    return {"samples_per_s": round(v, 1), "ms_per_step": round(elapsed / steps * 1000, 4),
            "vs_baseline": round(v / BASELINE_LSTM, 2),
            "config": f"Embedding(95812,32)+LSTM(32,32,L2)+fc4, T129, batch 32/GPU, Adam, fp32, dp{world}"}


def bench_mlp(args, rank, world, device):
    """distributed_multilayer_perceptron.py workload: 4-5-4-3 sigmoid MLP, batch 30/GPU, SGD."""
    import torch
    from sparkmi.models.mlp import MultilayerPerceptron
    from sparkmi.optim import SGD
    from sparkmi.parallel.ddp import DataParallel
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    fresh_model_state(5)
    model = MultilayerPerceptron((4, 5, 4, 3)).to(device).train()
    flat = FlatParams(model, shadow=False)
    opt = SGD(flat, lr=0.01)
    ddp = DataParallel(flat) if world > 1 else None
    # one executor: the whole step (forward, CE, backward, SGD) is ONE kernel launch; data-parallel:
    # forward + backward in one kernel (gradients to the flat buffer), the IPC all-reduce and SGD
    fused = (lambda m, o, x, y: m.fused_sgd_step(o, x, y)) if world == 1 else None
    fgrad = (lambda m, x, y: m.fused_grad_step(x, y)) if world > 1 else None
    # one executor, multi-step graphs: each run of `unroll` steps is ONE launch of the multi-step
    # kernel (parameters on chip between the steps)
    fsteps = (lambda m, o, bs: m.fused_sgd_steps(o, bs)) if world == 1 else None
    runner = StepRunner(model, lambda m, x, y: m.loss(x, y), opt, ddp, graph=device.type == "cuda" and args.graph != "off",
                        fused_step=fused, bind_inputs=True, fused_grad=fgrad, fused_steps=fsteps)
    g = torch.Generator().manual_seed(31 + rank)
    # 32 distinct batches: one cycle over them is one launch of the multi-step kernel (its capacity)
    batches = [(torch.rand(30, 4, generator=g).to(device) * 2 - 1, torch.randint(0, 3, (30,), generator=g).to(device))
               for _ in range(32)]
    steps = args.aux_steps
    elapsed, _ = time_steps(runner, batches, steps, max(args.warmup, 5), device, world)
    if ddp is not None:
        ddp.close()
    v = world * 30 * steps / elapsed
    return {"samples_per_s": round(v, 1), "ms_per_step": round(elapsed / steps * 1000, 4),
            "vs_baseline": round(v / BASELINE_MLP, 2), "config": f"MLP 4-5-4-3 sigmoid, batch 30/GPU, SGD, fp32, dp{world}"}


def bench_transformer(args, rank, world, device, dtype, zero=False):
    """One full training step of the BASELINE transformer at ``dtype`` ('fp32' = reference
    precision, or 'bf16' = bf16 activations/weights with fp32 master weights and fp32 accumulate)."""
    import torch
    from sparkmi.data.synthetic import copy_pairs, translation_pairs
    from sparkmi.models.transformer import Transformer, transformer_flops_per_sample
    from sparkmi.optim import Adam
    from sparkmi.parallel.ddp import DataParallel
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    fresh_model_state(1234)
    model = Transformer(d_model=512, ffn_hidden=1024, num_heads=8, drop_prob=0.1, num_layers=args.layers,
                        max_sequence_length=args.seq, src_vocab_size=args.vocab, tgt_vocab_size=args.vocab,
                        mask_mode="reference", seed=1234 + rank, dtype=dtype).to(device)
    model.train()
    flat = FlatParams(model, shadow=(dtype == "bf16" and device.type == "cuda"))
    opt = Adam(flat, lr=1e-3)
    ddp = DataParallel(flat, bucket_mb=args.bucket_mb, zero=zero) if world > 1 else None
    use_graph = args.graph != "off" and device.type == "cuda"
    # data-parallel: backward in several graphs (decoder, then encoder halves) so the finished
    # gradient buckets are all-reduced while the rest of the backward runs (sparkmi/train/runner.py)
    split_fn = (lambda m, s, t: m.training_step_split(s, t)) if (world > 1 and args.split and use_graph) else None
    runner = StepRunner(model, lambda m, s, t: m.training_step_loss(s, t), opt, ddp, graph=use_graph,
                        split_fn=split_fn)
    pool = 8
    if args.data == "copy":
        src, tgt = copy_pairs(pool * args.batch, args.seq, args.vocab, seed=100 + rank, device=device)
    else:
        src, tgt = translation_pairs(pool * args.batch, args.seq, args.vocab, args.vocab, seed=100 + rank,
                                     device=device)
    src = src.view(pool, args.batch, args.seq)
    tgt = tgt.view(pool, args.batch, args.seq)
    batches = [(src[i], tgt[i]) for i in range(pool)]
    losses = []
    elapsed, loss = time_steps(runner, batches, args.steps, args.warmup, device, world, record=losses)
    final_loss = float(loss.float().item()) if loss is not None else float("nan")
    in_sync = ranks_in_sync(flat, world)
    ar = time_allreduce(flat, device, world)
    comm = None
    if ddp is not None:
        comm = {"path": ddp.comm, "probe": ddp.comm_probe}
        ddp.close()
        if dtype == "fp32" and not zero:
            comm["paths"] = time_comm_paths(device, world, args.bucket_mb)
    value = world * args.batch * args.steps / elapsed
    tflops = transformer_flops_per_sample(args.layers, args.seq, args.vocab) * value / world / 1e12
    peak = 157.3 if dtype == "fp32" else 2500.0
    res = {"samples_per_s": round(value, 2), "ms_per_step": round(elapsed / args.steps * 1000, 3),
           "final_loss": round(final_loss, 4), "losses": [round(float(l), 4) for l in losses],
           # random data: src / tgt independent and uniform over V - 4 content tokens -> no model beats ln(V - 4)
           "loss_floor": round(math.log(args.vocab - 4), 4) if args.data == "random" else 0.0, "data": args.data,
           "model_tflops_per_gpu": round(tflops, 1),
           f"mfu_vs_{'157tf_fp32' if dtype == 'fp32' else '2.5pf_bf16'}_dense": round(tflops / peak, 3),
           "allreduce_ms": ar, "grad_bytes": flat.numel * 4, "dtype": dtype,
           "overlap": "finished buckets all-reduced under the rest of the backward" if split_fn else None,
           "hip_graph": use_graph, "zero1": bool(zero and world > 1), "comm": comm,
           "ranks_in_sync": in_sync}
    if dtype == "fp32":
        # the algorithm the step actually runs: 6 bf16 products per fp32 product
        res["mfu_vs_417tf_split3_ceiling"] = round(tflops / SPLIT_PEAK_TF, 3)
        res["mfu_vs_211tf_measured_split3_ceiling"] = round(tflops / SPLIT_MEASURED_TF, 3)
    else:
        res["mfu_vs_1268tf_measured_bf16_gemm"] = round(tflops / BF16_MEASURED_TF, 3)
    del runner, opt, flat, model, ddp, batches, src, tgt
    if device.type == "cuda":
        torch.cuda.empty_cache()
    return res


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: become the launcher (before importing anything that touches the GPU)
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    if args.device == "cpu":
        os.environ["SPARKMI_FORCE_CPU"] = "1"
    import torch
    from sparkmi.parallel import destroy, init_distributed
    rank, world, device = init_distributed()
    if args.dtype == "auto":
        dtypes = ["fp32", "bf16"] if device.type == "cuda" else ["fp32"]
    elif args.dtype == "both":
        dtypes = ["fp32", "bf16"]
    else:
        dtypes = [args.dtype]
    cnn = cnn32 = cnn_recipe = lstm = mlp = None

    def side(fn, *a):
        # an extra workload that raises must not take the headline down with it; reported as its
        # error.  Every rank learns whether ANY rank failed (one MAX all-reduce of a flag) and all
        # take the error branch together, so a rank that failed alone never walks into the next
        # workload's collectives while its peers are still inside this one's
        if args.model != "all":
            return fn(*a)
        out, err = None, None
        try:
            out = fn(*a)
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"[:300]
        if world > 1:
            import torch.distributed as dist
            flag = torch.tensor([1 if err else 0], dtype=torch.int32,
                                device=device if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            if int(flag.item()) and err is None:
                err = "failed on another rank"
        return {"error": err} if err else out
    if args.model in ("all", "cnn"):
        # BASELINE's CNN config is bf16 (Conv2d on matrix cores); the fp32 kernel is reported too
        cnn32 = side(bench_cnn, args, rank, world, device, "fp32")
        cnn = side(bench_cnn, args, rank, world, device, "bf16") if device.type == "cuda" else cnn32
        cnn_recipe = side(bench_cnn_recipe, args, rank, world, device, "bf16" if device.type == "cuda" else "fp32")
    if args.model in ("all", "aux") and not args.no_aux:
        lstm = side(bench_lstm, args, rank, world, device)
        mlp = side(bench_mlp, args, rank, world, device)
    if args.model == "aux":  # LSTM + MLP extras only (profiling)
        if rank == 0:
            print(json.dumps({"lstm": lstm, "mlp": mlp, "n_gpus": world}))
        destroy()
        return
    if args.model == "cnn":
        if rank == 0:
            print(json.dumps({"metric": "samples/sec (whole node) distributed_cnn at 1/2/4/8 MI355X",
                              "value": cnn["samples_per_s"], "unit": "samples/s", "n_gpus": world,
                              "steps": args.cnn_steps, "warmup": args.warmup, "ms_per_step": cnn["ms_per_step"],
                              "higher_is_better": True, "scaling": "weak", "vs_baseline": cnn["vs_baseline"],
                              "dtype": cnn["dtype"], "data": "synthetic",
                              "config": {"model": "FashionMNISTModel", "global_batch": cnn["global_batch"],
                                         "seq_len": None, "parallelism": f"dp{world}"}, "cnn": cnn,
                              "cnn_fp32": cnn32, "cnn_recipe_path": cnn_recipe}))
        destroy()
        return
    tr = {dt: bench_transformer(args, rank, world, device, dt) for dt in dtypes}
    head = tr[dtypes[0]]
    f32mfma = None
    if "fp32" in dtypes and device.type == "cuda" and not args.no_f32_compare:
        # the same fp32 step with every GEMM product on v_mfma_f32_32x32x2_f32 instead of the
        # exact-product bf16 split (both fp32 in / out / accumulate), for comparison
        from sparkmi import _native
        from sparkmi.ops import gemm as G
        C = _native.C()
        prev, prev_sp = C.gemm_f32_algo(-1), G.SP
        C.gemm_f32_algo(0)
        G.SP = False
        try:
            f32mfma = side(bench_transformer, args, rank, world, device, "fp32")
        finally:
            C.gemm_f32_algo(prev)
            G.SP = prev_sp
    zero1 = None
    if world > 1 and "fp32" in dtypes and not args.no_zero_compare:
        # ZeRO-1 beside the headline (reduce-scatter under the backward, sharded Adam, parameter
        # all-gather after it): measured at every N so the replicated-vs-sharded choice rests on data
        zero1 = side(bench_transformer, args, rank, world, device, "fp32", True)
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": head["samples_per_s"],
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(head["samples_per_s"] / BASELINE_TRANSFORMER, 2),
            "dtype": dtypes[0],
            "data": "synthetic (Multi30k-shaped token ids, HBM-resident); random-init weights",
            "config": {
                "model": f"transformer.py enc-dec L{args.layers} d512 h8 ffn1024 V{args.vocab}/{args.vocab}",
                "global_batch": world * args.batch,
                "seq_len": args.seq,
                "parallelism": f"dp{world}",
                "optimizer": "Adam lr1e-3 (fp32, fused HIP)",
                "mask_mode": "reference",
                "precision": (F32_PRECISION if dtypes[0] == "fp32"
                              else "bf16 activations, fp32 master weights + accumulate"),
                "baseline_ref": "BASELINE.md §2 transformer L6/S256 CPU proxy 4.79 samples/s",
            },
            "allreduce_ms": head["allreduce_ms"],
            "losses": head.get("losses"),
        }
        for dt in dtypes:
            out[f"transformer_{dt}"] = tr[dt]
        if f32mfma is not None:
            out["transformer_fp32_f32mfma"] = f32mfma
        if zero1 is not None:
            out["transformer_fp32_zero1"] = zero1
        if cnn is not None:
            out["cnn"] = cnn
            out["cnn_fp32"] = cnn32
            out["cnn_recipe_path"] = cnn_recipe
        if lstm is not None:
            out["extra"] = {"lstm": lstm, "mlp": mlp,
                            "aux_baseline_ref": "BASELINE.md §2 best CPU proxy: LSTM 1,365, MLP 130,476 samples/s"}
        print(json.dumps(out), flush=True)
    destroy()


if __name__ == "__main__":
    main()
