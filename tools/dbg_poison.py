"""Uninitialised-read hunt: fill the caching allocator's free blocks with NaN, then run the
concat-kv GPU-vs-CPU gradient comparison (both product algorithms); a kernel that reads memory
it never wrote turns the NaN into a mismatch."""
import os, sys, torch
sys.path.insert(0, os.getcwd())
from sparkmi import _native
import tests.test_f32_gpu as T
from sparkmi.data.synthetic import translation_pairs
from sparkmi.utils.flat import FlatParams
C = _native.C()

def poison():
    bufs = []
    for mb in (1, 2, 4, 8, 16, 32, 64, 128) * 4:
        bufs.append(torch.full((mb * 262144,), float("nan"), device="cuda"))
    torch.cuda.synchronize()
    del bufs

for algo in (6, 0):
    C.gemm_f32_algo(algo)
    for L in (3, 2):
        poison()
        mc, mg = T._pair(L=L)
        mc.train(); mg.train()
        fc, fg = FlatParams(mc), FlatParams(mg, shadow=False)
        src, tgt = translation_pairs(4, 32, 96, 96, seed=3)
        fg.zero_grad()
        lc = mc.training_step_loss(src, tgt)
        lg = mg.training_step_loss(src.to('cuda'), tgt.to('cuda'))
        lc.backward(); lg.backward(); torch.cuda.synchronize()
        bad = []
        for (n, pc), (_, pg) in zip(mc.named_parameters(), mg.named_parameters()):
            g = pg.grad.cpu().double()
            rel = float((g - pc.grad.double()).norm() / (pc.grad.double().norm() + 1e-12))
            if not (rel < 1e-4): bad.append((n, rel))
        print("algo", algo, "L", L, "loss", float(lc), float(lg), "bad", len(bad), bad[:8], flush=True)
