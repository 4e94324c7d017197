"""In-process A/B of the fused CNN step (bound batches, multi-step graphs, like bench.py's CNN
bench): `python tools/ab_cnn.py MODULE:ATTR=v1,v2 [--dtype bf16|fp32] [--rounds R]` times the step
with the module constant set to each value in turn (e.g. sparkmi.ops.cnn:WGRAD_HELPERS=1,0)."""
import argparse
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def run(dtype, steps=400):
    import bench
    from sparkmi.data.synthetic import fashion_mnist_like
    from sparkmi.models.cnn import FashionMNISTModel
    from sparkmi.optim import SGD
    from sparkmi.train.runner import StepRunner
    from sparkmi.utils.flat import FlatParams
    torch.manual_seed(0)
    model = FashionMNISTModel(1, 10, 10, dtype=dtype).cuda().train()
    flat = FlatParams(model, shadow=False)
    opt = SGD(flat, lr=0.01)
    runner = StepRunner(model, lambda m, x, y: m.loss(x, y), opt, None, graph=True,
                        fused_step=lambda m, o, x, y: m.fused_sgd_step(o, x, y), bind_inputs=True)
    x, y = fashion_mnist_like(32 * 16, seed=3)
    x, y = x.cuda(), y.cuda()
    batches = [(x[i * 32:(i + 1) * 32], y[i * 32:(i + 1) * 32]) for i in range(16)]
    elapsed, _ = bench.time_steps(runner, batches, steps, 5, torch.device("cuda"), 1)
    return elapsed / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("spec")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    target, vals = a.spec.split("=")
    mod, attr = target.split(":")
    m = importlib.import_module(mod)
    res = {}
    for _ in range(a.rounds):
        for v in vals.split(","):
            setattr(m, attr, type(getattr(m, attr))(int(v)) if isinstance(getattr(m, attr), (bool, int)) else v)
            ms = run(a.dtype)
            res.setdefault(v, []).append(round(ms, 4))
            print(json.dumps({attr: v, "ms_per_step": round(ms, 4)}), flush=True)
    for v, r in res.items():
        print(json.dumps({attr: v, "ms_per_step_min": min(r), "all": r}))


if __name__ == "__main__":
    main()
