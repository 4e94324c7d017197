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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="transformer", choices=["transformer"])
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=256)
    ap.add_argument("--layers", type=int, default=6)
    ap.add_argument("--vocab", type=int, default=10000)
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"])
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    return ap.parse_args()


def main():
    args = parse()
    from sparkmi.parallel import barrier, init_distributed
    from sparkmi.parallel.ddp import DataParallel
    rank, world, device = init_distributed()
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
    use_graph = {"on": True, "off": False, "auto": world == 1}[args.graph] and device.type == "cuda"
    runner = StepRunner(model, lambda m, s, t: m.training_step_loss(s, t), opt, ddp, graph=use_graph)
    pool = 8
    src, tgt = translation_pairs(pool * args.batch, args.seq, args.vocab, args.vocab, seed=100 + rank, device=device)
    src = src.view(pool, args.batch, args.seq)
    tgt = tgt.view(pool, args.batch, args.seq)

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize()

    loss = None
    for i in range(args.warmup):
        loss = runner.step(src[i % pool], tgt[i % pool])
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = runner.step(src[i % pool], tgt[i % pool])
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss.float().item()) if loss is not None else float("nan")
    value = world * args.batch * args.steps / elapsed
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
                "baseline_ref": "BASELINE.md §2 transformer L6/S256 CPU proxy 4.79 samples/s",
                "final_loss": round(final_loss, 4),
            },
        }
        print(json.dumps(out), flush=True)
    from sparkmi.parallel import destroy
    destroy()


if __name__ == "__main__":
    main()
