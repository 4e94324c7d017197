#!/usr/bin/env python3
"""In-process A/B of transformer-step variants (module-level switches), interleaved rounds so clock
drift hits every variant alike.  Usage (GPU box):
    python tools/ab_step.py --dtype fp32 --rounds 2 'sparkmi.models.transformer:WGRAD_FLUSH_LAYERS=none,encoder,all'
Each spec is module:attribute=v1,v2,... (a module attribute) or C:function=v1,v2,... (a setter of
the native extension, e.g. C:gemm_sp_wg_tm=0,16,128); values are parsed as Python literals."""
import argparse
import ast
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("spec")
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    modname, rest = a.spec.split(":")
    attr, vals = rest.split("=")
    if modname == "C":
        from sparkmi import _native
        mod = None
        setter = getattr(_native.C(), attr)
    else:
        mod = importlib.import_module(modname)
        setter = lambda v: setattr(mod, attr, v)  # noqa: E731
    values = []
    for v in vals.split(","):
        try:
            values.append(ast.literal_eval(v))
        except (ValueError, SyntaxError):
            values.append(v)
    import torch
    from sparkmi.parallel import init_distributed
    rank, world, device = init_distributed()
    args = bench.parse(["--steps", str(a.steps), "--warmup", "5"])
    res = {str(v): [] for v in values}
    for _ in range(a.rounds):
        for v in values:
            setter(v)
            r = bench.bench_transformer(args, rank, world, device, a.dtype)
            res[str(v)].append(r["ms_per_step"])
            print(json.dumps({attr: v, "ms_per_step": r["ms_per_step"]}), flush=True)
    for v, ms in res.items():
        print(json.dumps({attr: v, "ms_per_step_min": min(ms), "all": ms}), flush=True)


if __name__ == "__main__":
    main()
