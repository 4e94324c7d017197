"""Stock PyTorch-ROCm comparison point for the flagship benchmark.

The same encoder-decoder Transformer shape as bench.py (6+6 layers, d_model 512, 8 heads, ffn
1024, seq 256, vocab 10k/10k, post-LN blocks, dropout 0.1, batch 32, Adam lr 1e-3, token
cross-entropy) written with plain torch.nn / torch.nn.functional ops — hipBLASLt GEMMs,
PyTorch's fused SDPA, native LayerNorm, fused Adam — under bf16 autocast with fp32 master
weights, eager mode.  It is an independent implementation of the architecture (not sparkmi,
not the reference script); it exists only to put sparkmi's number next to what stock PyTorch
does on the same MI355X.  Prints one JSON line.

    python tools/bench_torch_baseline.py [--steps 20 --warmup 5 --batch 32 --seq 256 --layers 6]
    python tools/bench_torch_baseline.py --model cnn|lstm|mlp [--steps 200]

``--model cnn|lstm|mlp``: the other three reference workloads in stock torch.nn (MIOpen convs,
cuDNN-style fused nn.LSTM, nn.Linear MLP), same shapes/optimizers as bench.py's extras, eager.
"""
import argparse
import json
import math
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class Block(nn.Module):
    def __init__(self, d, heads, ffn, p, cross):
        super().__init__()
        self.heads = heads
        self.qkv = nn.Linear(d, 3 * d)
        self.out = nn.Linear(d, d)
        self.n1 = nn.LayerNorm(d)
        self.cross = cross
        if cross:
            self.q = nn.Linear(d, d)
            self.kv = nn.Linear(d, 2 * d)
            self.cout = nn.Linear(d, d)
            self.n2 = nn.LayerNorm(d)
        self.f1 = nn.Linear(d, ffn)
        self.f2 = nn.Linear(ffn, d)
        self.n3 = nn.LayerNorm(d)
        self.p = p

    def _split(self, x):
        b, s, d = x.shape
        return x.view(b, s, self.heads, d // self.heads).transpose(1, 2)

    def _merge(self, x):
        b, h, s, dh = x.shape
        return x.transpose(1, 2).reshape(b, s, h * dh)

    def forward(self, y, enc=None, causal=False):
        q, k, v = self.qkv(y).chunk(3, dim=-1)
        a = F.scaled_dot_product_attention(self._split(q), self._split(k), self._split(v), is_causal=causal)
        y = self.n1(y + F.dropout(self.out(self._merge(a)), self.p, self.training))
        if self.cross:
            k, v = self.kv(enc).chunk(2, dim=-1)
            a = F.scaled_dot_product_attention(self._split(self.q(y)), self._split(k), self._split(v))
            y = self.n2(y + F.dropout(self.cout(self._merge(a)), self.p, self.training))
        f = self.f2(F.dropout(F.relu(self.f1(y)), self.p, self.training))
        return self.n3(y + F.dropout(f, self.p, self.training))


class Seq2Seq(nn.Module):
    def __init__(self, layers, d, heads, ffn, vs, vt, seq, p=0.1):
        super().__init__()
        self.se = nn.Embedding(vs, d)
        self.te = nn.Embedding(vt, d)
        pos = torch.arange(seq).float()[:, None]
        div = torch.exp(torch.arange(0, d, 2).float() * (-math.log(10000.0) / d))
        pe = torch.zeros(seq, d)
        pe[:, 0::2] = torch.sin(pos * div)
        pe[:, 1::2] = torch.cos(pos * div)
        self.register_buffer("pe", pe)
        self.enc = nn.ModuleList([Block(d, heads, ffn, p, False) for _ in range(layers)])
        self.dec = nn.ModuleList([Block(d, heads, ffn, p, True) for _ in range(layers)])
        self.head = nn.Linear(d, vt)
        self.p = p

    def forward(self, src, tgt):
        x = F.dropout(self.se(src) + self.pe, self.p, self.training)
        for blk in self.enc:
            x = blk(x)
        y = F.dropout(self.te(tgt) + self.pe, self.p, self.training)
        for blk in self.dec:
            y = blk(y, x, causal=True)
        return self.head(y)


def _time(step, warmup, steps):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    return time.perf_counter() - t0, loss


def small_model(a):
    """distributed_cnn.py / distributed_lstm.py / distributed_multilayer_perceptron.py shapes."""
    dev = torch.device("cuda")
    torch.manual_seed(0)
    if a.model == "cnn":
        B = 32
        m = nn.Sequential(nn.Conv2d(1, 10, 3, padding=1), nn.ReLU(), nn.Conv2d(10, 10, 3, padding=1), nn.ReLU(),
                          nn.MaxPool2d(2), nn.Conv2d(10, 10, 3, padding=1), nn.ReLU(), nn.Conv2d(10, 10, 3, padding=1),
                          nn.ReLU(), nn.MaxPool2d(2), nn.Flatten(), nn.Linear(490, 10)).to(dev)
        opt = torch.optim.SGD(m.parameters(), lr=0.01)
        x = torch.rand(B, 1, 28, 28, device=dev)
        y = torch.randint(0, 10, (B,), device=dev)
        fwd = lambda: F.cross_entropy(m(x), y)  # noqa: E731
    elif a.model == "lstm":
        B, T, V = 32, 129, 95812

        class L(nn.Module):
            def __init__(self):
                super().__init__()
                self.emb = nn.Embedding(V, 32, padding_idx=7)
                self.lstm = nn.LSTM(32, 32, num_layers=2, batch_first=True, dropout=0.5)
                self.fc = nn.Linear(32, 4)

            def forward(self, t):
                h, _ = self.lstm(self.emb(t))
                return self.fc(h)

        m = L().to(dev)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        x = torch.randint(0, V, (B, T), device=dev)
        y = torch.randint(0, 4, (B,), device=dev)
        fwd = lambda: F.cross_entropy(m(x)[:, -1, :], y)  # noqa: E731
    else:
        B = 30
        m = nn.Sequential(nn.Linear(4, 5), nn.Sigmoid(), nn.Linear(5, 4), nn.Sigmoid(), nn.Linear(4, 3)).to(dev)
        opt = torch.optim.SGD(m.parameters(), lr=0.01)
        x = torch.rand(B, 4, device=dev) * 2 - 1
        y = torch.randint(0, 3, (B,), device=dev)
        fwd = lambda: F.cross_entropy(m(x), y)  # noqa: E731
    m.train()

    def step():
        opt.zero_grad(set_to_none=True)
        loss = fwd()
        loss.backward()
        opt.step()
        return loss

    dt, loss = _time(step, a.warmup, a.steps)
    print(json.dumps({"metric": f"stock PyTorch eager {a.model} samples/s (1 GPU)", "value": round(B * a.steps / dt, 1),
                      "ms_per_step": round(dt / a.steps * 1000, 4), "batch": B, "dtype": "fp32",
                      "final_loss": round(float(loss), 4), "torch": torch.__version__}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="transformer", choices=["transformer", "cnn", "lstm", "mlp"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=256)
    ap.add_argument("--layers", type=int, default=6)
    ap.add_argument("--vocab", type=int, default=10000)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                    help="bf16 autocast (fp32 master) or plain fp32 (the reference precision)")
    a = ap.parse_args()
    if a.model != "transformer":
        return small_model(a)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = Seq2Seq(a.layers, 512, 8, 1024, a.vocab, a.vocab, a.seq).to(dev).train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, fused=True)
    src = torch.randint(1, a.vocab, (a.batch, a.seq), device=dev)
    tgt = torch.randint(1, a.vocab, (a.batch, a.seq), device=dev)

    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.dtype == "bf16"):
            logits = m(src, tgt)
            loss = F.cross_entropy(logits.float().view(-1, a.vocab), tgt.view(-1), ignore_index=0)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"metric": "stock PyTorch eager transformer samples/s (1 GPU)", "value": round(a.batch * a.steps / dt, 2),
                      "ms_per_step": round(dt / a.steps * 1000, 3), "batch": a.batch, "seq": a.seq, "layers": a.layers,
                      "dtype": "bf16 autocast, fp32 master" if a.dtype == "bf16" else "fp32",
                      "final_loss": round(float(loss), 4),
                      "torch": torch.__version__}))


if __name__ == "__main__":
    main()
