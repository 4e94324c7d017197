#!/usr/bin/env python3
"""Headline benchmark: whole-node training samples/sec of the reference workloads on MI355X.

Flagship = the BASELINE.json transformer config: encoder-decoder Transformer (transformer.py),
6 layers, d_model 512, 8 heads, ffn 1024, seq 256, vocab 10k/10k, batch 32 per GPU, Adam
lr 1e-3, dropout 0.1, reference mask semantics, bf16 compute / fp32 master weights — a full
training step (forward, masked token CE, backward, gradient all-reduce, optimizer) per
iteration, synthetic Multi30k-shaped data resident in HBM, random-init weights.

Contract: ``python bench.py --gpus N --steps K --warmup W``; multi-GPU runs are launched by
torch.distributed.run (one rank per GPU, RCCL).  W untimed warm-up steps, then K steps timed
between barrier+synchronize on both sides; the MAX elapsed over ranks is used; rank 0 prints
one JSON line.  ``value`` = whole-job samples/s = N * batch * K / max_elapsed (weak scaling).
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# transformer L6/S256/B32 CPU proxy, best whole-node figure (1 proc x 8 threads)
BASELINE_TRANSFORMER = 4.79
BASELINE_CNN = 5655.0
BASELINE_LSTM = 1365.0    # 1 proc x 8 threads
BASELINE_MLP = 130476.0   # world 1, 1 thread


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="all", choices=["all", "transformer", "cnn", "aux"])
    ap.add_argument("--aux-steps", type=int, default=100, help="timed steps of the LSTM / MLP extras")
    ap.add_argument("--cnn-batch", type=int, default=32)
    ap.add_argument("--cnn-steps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=256)
    ap.add_argument("--layers", type=int, default=6)
    ap.add_argument("--vocab", type=int, default=10000)
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"])
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--split", type=int, default=1, help="two-graph backward with overlapped all-reduce (DP)")
    return ap.parse_args()


def transformer_flops_per_sample(layers, seq, vocab, d=512, ffn=1024):
    """Matmul FLOPs of one training sample (forward + backward = 3x forward): per token, each
    encoder layer's QKV / out-projection / FFN GEMMs, each decoder layer's self QKV / out,
    cross Q / KV / out and FFN GEMMs, the vocab projection, plus QK^T and PV of the 3 attention
    sites per layer pair (63.4 GFLOP at L6 S256 V10k)."""
    enc = 2 * d * (3 * d + d + 2 * ffn)
    dec = 2 * d * (3 * d + d + d + 2 * d + d + 2 * ffn)
    attn = 3 * 4 * seq * d
    per_token = layers * (enc + dec + attn) + 2 * d * vocab
    return 3 * per_token * seq


def time_steps(runner, batches, steps, warmup, device, world):
    from sparkmi.parallel import barrier
    sync = (lambda: torch.cuda.synchronize()) if device.type == "cuda" else (lambda: None)
    n = len(batches)
    loss = None
    for i in range(warmup):
        loss = runner.step(*batches[i % n])
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        loss = runner.step(*batches[i % n])
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, loss


def bench_cnn(args, rank, world, device):
    """distributed_cnn.py workload: FashionMNISTModel, batch 32/GPU, SGD lr 0.01, mean CE."""
    from sparkmi.data.synthetic import fashion_mnist_like
    from sparkmi.models.cnn import FashionMNISTModel
    from sparkmi.optim import SGD
    from sparkmi.parallel.ddp import DataParallel
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    torch.manual_seed(4321)
    model = FashionMNISTModel(1, 10, 10).to(device).train()
    flat = FlatParams(model)
    opt = SGD(flat, lr=0.01)
    ddp = DataParallel(flat) if world > 1 else None
    use_graph = device.type == "cuda" and args.graph != "off"
    runner = StepRunner(model, lambda m, x, y: m.loss(x, y), opt, ddp, graph=use_graph)
    imgs, labels = fashion_mnist_like(16 * args.cnn_batch, seed=7 + rank, device=device)
    batches = [(imgs[i * args.cnn_batch:(i + 1) * args.cnn_batch], labels[i * args.cnn_batch:(i + 1) * args.cnn_batch])
               for i in range(16)]
    elapsed, loss = time_steps(runner, batches, args.cnn_steps, max(args.warmup, 5), device, world)
    if ddp is not None:
        ddp.close()
    return world * args.cnn_batch * args.cnn_steps / elapsed, elapsed / args.cnn_steps * 1000, float(loss)


def bench_lstm(args, rank, world, device):
    """distributed_lstm.py workload: Embedding(V~95.8k, 32) -> LSTM(32, 32, 2 layers, dropout 0.5)
    -> fc(4) at every step, CE on the last step; batch 32/GPU, T = 129, Adam lr 1e-3."""
    from sparkmi.models.lstm import LSTM
    from sparkmi.optim import Adam
    from sparkmi.parallel.ddp import DataParallel
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    V, B, T = 95812, 32, 129
    torch.manual_seed(11)
    model = LSTM(V, 32, 32, 4, num_layers=2, padding_idx=7).to(device).train()
    flat = FlatParams(model, shadow=False)
    opt = Adam(flat, lr=1e-3)
    ddp = DataParallel(flat) if world > 1 else None
    runner = StepRunner(model, lambda m, x, y: m.loss(x, y)[0], opt, ddp, graph=device.type == "cuda" and args.graph != "off")
    g = torch.Generator().manual_seed(21 + rank)
    batches = [(torch.randint(0, V, (B, T), generator=g).to(device), torch.randint(0, 4, (B,), generator=g).to(device))
               for _ in range(8)]
    steps = args.aux_steps
    elapsed, _ = time_steps(runner, batches, steps, max(args.warmup, 5), device, world)
    if ddp is not None:
        ddp.close()
    return world * B * steps / elapsed, elapsed / steps * 1000


def bench_mlp(args, rank, world, device):
    """distributed_multilayer_perceptron.py workload: 4-5-4-3 sigmoid MLP, batch 30/GPU, SGD."""
    from sparkmi.models.mlp import MultilayerPerceptron
    from sparkmi.optim import SGD
    from sparkmi.parallel.ddp import DataParallel
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    torch.manual_seed(5)
    model = MultilayerPerceptron((4, 5, 4, 3)).to(device).train()
    flat = FlatParams(model, shadow=False)
    opt = SGD(flat, lr=0.01)
    ddp = DataParallel(flat) if world > 1 else None
    runner = StepRunner(model, lambda m, x, y: m.loss(x, y), opt, ddp, graph=device.type == "cuda" and args.graph != "off")
    g = torch.Generator().manual_seed(31 + rank)
    batches = [(torch.rand(30, 4, generator=g).to(device) * 2 - 1, torch.randint(0, 3, (30,), generator=g).to(device))
               for _ in range(8)]
    steps = args.aux_steps
    elapsed, _ = time_steps(runner, batches, steps, max(args.warmup, 5), device, world)
    if ddp is not None:
        ddp.close()
    return world * 30 * steps / elapsed, elapsed / steps * 1000


def main():
    args = parse()
    from sparkmi.parallel import barrier, init_distributed
    from sparkmi.parallel.ddp import DataParallel
    rank, world, device = init_distributed()
    cnn = lstm = mlp = None
    if args.model in ("all", "cnn"):
        cnn = bench_cnn(args, rank, world, device)
    if args.model in ("all", "aux"):
        lstm = bench_lstm(args, rank, world, device)
        mlp = bench_mlp(args, rank, world, device)
    if args.model == "aux":  # LSTM + MLP extras only (profiling)
        if rank == 0:
            print(json.dumps({"lstm_samples_per_s": round(lstm[0], 1), "lstm_ms_per_step": round(lstm[1], 4),
                              "mlp_samples_per_s": round(mlp[0], 1), "mlp_ms_per_step": round(mlp[1], 4),
                              "n_gpus": world}))
        return
    if args.model == "cnn":
        if rank == 0:
            v, ms, l = cnn
            print(json.dumps({"metric": "samples/sec (whole node) distributed_cnn at 1/2/4/8 MI355X", "value": round(v, 1),
                              "unit": "samples/s", "n_gpus": world, "steps": args.cnn_steps, "warmup": args.warmup,
                              "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
                              "vs_baseline": round(v / BASELINE_CNN, 2), "dtype": "fp32", "data": "synthetic",
                              "config": {"model": "FashionMNISTModel", "global_batch": world * args.cnn_batch,
                                         "seq_len": None, "parallelism": f"dp{world}", "final_loss": round(l, 4)}}))
        return
    torch.manual_seed(1234)
    from sparkmi.models.transformer import Transformer
    from sparkmi.optim import Adam
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    from sparkmi.data.synthetic import translation_pairs

    model = Transformer(d_model=512, ffn_hidden=1024, num_heads=8, drop_prob=0.1, num_layers=args.layers,
                        max_sequence_length=args.seq, src_vocab_size=args.vocab, tgt_vocab_size=args.vocab,
                        mask_mode="reference", seed=1234 + rank).to(device)
    model.train()
    flat = FlatParams(model)
    opt = Adam(flat, lr=1e-3)
    ddp = DataParallel(flat, bucket_mb=args.bucket_mb) if world > 1 else None
    use_graph = args.graph != "off" and device.type == "cuda"
    # data-parallel: backward in two graphs (decoder, then encoder) so the decoder's gradient
    # buckets are all-reduced while the encoder backward runs (sparkmi/train/runner.py)
    split_fn = (lambda m, s, t: m.training_step_split(s, t)) if (world > 1 and args.split) else None
    runner = StepRunner(model, lambda m, s, t: m.training_step_loss(s, t), opt, ddp, graph=use_graph,
                        split_fn=split_fn)
    pool = 8
    src, tgt = translation_pairs(pool * args.batch, args.seq, args.vocab, args.vocab, seed=100 + rank, device=device)
    src = src.view(pool, args.batch, args.seq)
    tgt = tgt.view(pool, args.batch, args.seq)

    batches = [(src[i], tgt[i]) for i in range(pool)]
    elapsed, loss = time_steps(runner, batches, args.steps, args.warmup, device, world)
    final_loss = float(loss.float().item()) if loss is not None else float("nan")
    value = world * args.batch * args.steps / elapsed
    tflops = transformer_flops_per_sample(args.layers, args.seq, args.vocab) * value / world / 1e12
    if rank == 0:
        out = {
            "metric": "samples/sec (whole node) distributed_cnn + transformer at 1/2/4/8 MI355X",
            "value": round(value, 2),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1000, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_TRANSFORMER, 2),
            "dtype": "bf16",
            "data": "synthetic (Multi30k-shaped token ids, HBM-resident); random-init weights",
            "config": {
                "model": f"transformer.py enc-dec L{args.layers} d512 h8 ffn1024 V{args.vocab}/{args.vocab}",
                "global_batch": world * args.batch,
                "seq_len": args.seq,
                "parallelism": f"dp{world}",
                "optimizer": "Adam lr1e-3 (fp32 master, fused HIP)",
                "mask_mode": "reference",
                "hip_graph": use_graph,
                "overlap": "decoder buckets all-reduced under the encoder backward" if split_fn else None,
                "baseline_ref": "BASELINE.md §2 transformer L6/S256 CPU proxy 4.79 samples/s",
                "final_loss": round(final_loss, 4),
                "model_tflops_per_gpu": round(tflops, 1),
                "mfu_vs_2.5pf_dense_bf16": round(tflops / 2500.0, 3),
            },
        }
        if cnn is not None:
            out["extra"] = {"cnn_samples_per_s": round(cnn[0], 1), "cnn_ms_per_step": round(cnn[1], 4),
                            "cnn_vs_baseline": round(cnn[0] / BASELINE_CNN, 2),
                            "cnn_config": f"FashionMNISTModel fp32 fused HIP kernel, batch {args.cnn_batch}/GPU, "
                                          f"SGD lr0.01, dp{world}, {args.cnn_steps} steps",
                            "cnn_baseline_ref": "BASELINE.md §2 CNN CPU proxy 5,655 samples/s (1 proc x 8 threads)"}
            if lstm is not None:
                out["extra"].update({
                    "lstm_samples_per_s": round(lstm[0], 1), "lstm_ms_per_step": round(lstm[1], 4),
                    "lstm_vs_baseline": round(lstm[0] / BASELINE_LSTM, 2),
                    "lstm_config": f"Embedding(95812,32)+LSTM(32,32,L2)+fc4, T129, batch 32/GPU, Adam, fp32, dp{world}",
                    "mlp_samples_per_s": round(mlp[0], 1), "mlp_ms_per_step": round(mlp[1], 4),
                    "mlp_vs_baseline": round(mlp[0] / BASELINE_MLP, 2),
                    "mlp_config": f"MLP 4-5-4-3 sigmoid, batch 30/GPU, SGD, fp32, dp{world}",
                    "aux_baseline_ref": "BASELINE.md §2 best CPU proxy: LSTM 1,365, MLP 130,476 samples/s"})
        print(json.dumps(out), flush=True)
    from sparkmi.parallel import destroy
    destroy()


if __name__ == "__main__":
    main()
