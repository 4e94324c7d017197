#!/usr/bin/env python3
"""Per-GEMM-class rate table of one training step from a rocprofv3 rocpd database: calls grouped
by kernel template and workgroup count (= output tile count, which with the model's K fixes the
shape), mean / min microseconds, and the achieved rate for the shapes given on the command line
as name-substring:wgs=M,N,K[/label] (FLOPs 2 M N K per call; fp32 classes also as bf16-plane
equivalent: 6 products per fp32 product).
Usage: python tools/gemm_classes.py run_results.db [--marker multi_copy_kernel] [--steps 4] [shape specs...]"""
import collections
import re
import sqlite3
import sys


def main():
    args = sys.argv[1:]
    db = args.pop(0)
    marker, steps = "multi_copy_kernel", 4
    if "--marker" in args:
        i = args.index("--marker"); marker = args[i + 1]; del args[i:i + 2]
    if "--steps" in args:
        i = args.index("--steps"); steps = int(args[i + 1]); del args[i:i + 2]
    shapes = {}
    for s in args:  # e.g. "gemm_sp_kernel<8, false, false, 1, 1>:256=8192,512,512/fwd N512"
        key, rest = s.rsplit(":", 1)
        wgs, mnk = rest.split("=")
        label = ""
        if "/" in mnk:
            mnk, label = mnk.split("/", 1)
        shapes[(key, int(wgs))] = (tuple(int(float(x)) for x in mnk.split(",")), label)
    c = sqlite3.connect(db)
    rows = c.execute("select name, grid_x, workgroup_x, end - start from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if marker in r[0]]
    lo, hi = marks[-steps - 1], marks[-1]
    agg = collections.defaultdict(list)
    for name, gx, wx, dur in rows[lo:hi]:
        n = re.sub(r"\(.*", "", name.replace("void ", ""))
        if "gemm" in n:
            agg[(n, gx // wx)].append(dur / 1e3)
    print(f"{'kernel':46s} {'wgs':>5s} {'n/step':>6s} {'mean_us':>8s} {'min_us':>7s} {'ms/step':>8s}  shape / rate at min (mean)")
    tot = 0.0
    for (n, w), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        tot += sum(v) / steps
        line = f"{n:46s} {w:5d} {len(v) / steps:6.1f} {sum(v) / len(v):8.1f} {min(v):7.1f} {sum(v) / steps:8.3f}"
        for (key, wgs), ((M, N, K), label) in shapes.items():
            if key in n and wgs == w:
                fl = 2.0 * M * N * K
                tf_min, tf_mean = fl / (min(v) * 1e-6) / 1e12, fl / (sum(v) / len(v) * 1e-6) / 1e12
                eq = " x6 = %.2f (%.2f) PF bf16-eq" % (6 * tf_min / 1e3, 6 * tf_mean / 1e3) if "sp" in n else ""
                line += f"  {label} {M}x{N}x{K}: {tf_min:.0f} ({tf_mean:.0f}) TF{eq}"
        print(line)
    print(f"total GEMM kernel time per step: {tot / 1e3:.3f} ms (kernel time, overlapped queues summed)")


if __name__ == "__main__":
    main()
