"""Every kernel call of one training step, in launch order, from a rocprofv3 rocpd database:
duration, grid / workgroup size, and the running total — the per-call view that
tools/step_timeline.py's per-family table hides (which GEMM shape is slow, not just which kernel).
Usage: python tools/step_calls.py gpurun_out/prof/run_results.db [--marker adam_kernel] [--step -1]
"""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="adam_kernel")
    ap.add_argument("--step", type=int, default=-1, help="which step (python index over the marker-delimited steps)")
    ap.add_argument("--abs", action="store_true", help="print start / end (us from the step's first kernel) instead")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)").fetchall()]
    want = ["name", "start", "end"]
    extra = [x for x in ("grid_size_x", "grid_size_y", "grid_size_z", "workgroup_size_x", "grid_x", "grid_y", "grid_z", "workgroup_x", "queue_id") if x in cols]
    rows = c.execute(f"select {', '.join(want + extra)} from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if r[0].removeprefix("void ").startswith(a.marker)]
    steps = list(zip(marks[:-1], marks[1:]))
    lo, hi = steps[a.step]
    tot = 0.0
    t0 = rows[lo + 1][1]
    for r in rows[lo + 1:hi + 1]:
        name = re.sub(r"\(.*", "", re.sub(r"^void ", "", r[0]))[:60]
        us = (r[2] - r[1]) / 1e3
        tot += us
        dims = " ".join(str(v) for v in r[3:])
        if a.abs:
            print(f"{(r[1] - t0) / 1e3:9.1f} {(r[2] - t0) / 1e3:9.1f} {us:8.1f}  {name:60s} {dims}")
        else:
            print(f"{us:9.1f} {tot:10.1f}  {name:60s} {dims}")


if __name__ == "__main__":
    main()
