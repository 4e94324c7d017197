import os, sys, torch
sys.path.insert(0, os.getcwd())
sys.argv = [sys.argv[0]]
from sparkmi import _native
from sparkmi.ops import _grad
import tests.test_f32_gpu as T
from sparkmi.data.synthetic import translation_pairs
from sparkmi.utils.flat import FlatParams
C = _native.C()
for algo in (6, 0):
    C.gemm_f32_algo(algo)
    for ov in (False, True):
        _grad.WGRAD_OVERLAP = ov
        mc, mg = T._pair(L=3)
        mc.train(); mg.train()
        fc, fg = FlatParams(mc), FlatParams(mg, shadow=False)
        src, tgt = translation_pairs(4, 32, 96, 96, seed=3)
        fg.zero_grad()
        lc = mc.training_step_loss(src, tgt)
        lg = mg.training_step_loss(src.to('cuda'), tgt.to('cuda'))
        lc.backward(); lg.backward(); torch.cuda.synchronize()
        bad = []
        for (n, pc), (_, pg) in zip(mc.named_parameters(), mg.named_parameters()):
            rel = float((pg.grad.cpu().double() - pc.grad.double()).norm() / (pc.grad.double().norm() + 1e-12))
            if rel > 1e-4: bad.append((n, round(rel, 6)))
        print("algo", algo, "overlap", ov, "bad", len(bad), bad[:6], flush=True)
