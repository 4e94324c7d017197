"""Per-step timeline from a rocprofv3 kernel-trace database (rocpd SQLite).

Splits the trace into training steps at each optimizer launch (``adam_kernel`` / ``sgd_kernel``
by default), and for the last ``--steps`` steps reports: wall span, GPU-busy time (union of all
kernels), idle gaps, busy time per HW queue (main vs side stream), and a per-kernel-family table
of time on each queue.  Usage:
    python tools/step_timeline.py gpurun_out/prof/run_results.db [--steps 5] [--marker adam_kernel]
"""
import argparse
import collections
import re
import sqlite3


def family(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"^void ", "", n)
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--marker", default="adam_kernel")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, queue_id, stream_id from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if r[0].removeprefix("void ").startswith(a.marker)]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"only {len(marks)} marker kernels found")
    lo, hi = marks[-a.steps - 1], marks[-1]
    seg = rows[lo + 1:hi + 1]
    t0, t1 = rows[lo][2], seg[-1][2]
    wall = (t1 - t0) / a.steps
    # union of busy intervals
    iv = sorted((s, e) for _, s, e, _, _ in seg)
    busy, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None:
            cs, ce = s, e
        elif s <= ce:
            ce = max(ce, e)
        else:
            busy += ce - cs
            cs, ce = s, e
    busy += ce - cs
    per_q = collections.defaultdict(int)
    fam = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for n, s, e, q, st in seg:
        per_q[q] += e - s
        fam[family(n)][q] += (e - s)
        cnt[family(n)] += 1
    qs = sorted(per_q, key=lambda q: -per_q[q])
    print(f"steps {a.steps}: wall {wall / 1e6:.3f} ms/step, GPU busy (union) {busy / a.steps / 1e6:.3f} ms/step, "
          f"idle {(wall - busy / a.steps) / 1e6:.3f} ms/step, kernels/step {len(seg) / a.steps:.0f}")
    for q in qs:
        print(f"  queue {q}: busy {per_q[q] / a.steps / 1e6:.3f} ms/step")
    print(f"{'kernel family':70s} {'n/step':>7s} " + " ".join(f"{'q' + str(q) + ' ms':>9s}" for q in qs))
    for f in sorted(fam, key=lambda f: -sum(fam[f].values())):
        print(f"{f:70s} {cnt[f] / a.steps:7.1f} " + " ".join(f"{fam[f][q] / a.steps / 1e6:9.3f}" for q in qs))
    gaps(rows, marks[-2], marks[-1])


def gaps(rows, lo, hi, top=12):
    """Idle intervals (no kernel running on any queue) inside one step, largest first."""
    seg = sorted(rows[lo + 1:hi + 1], key=lambda r: r[1])
    cur_end, prev, out = rows[lo][2], rows[lo][0], []
    for n, s, e, _, _ in seg:
        if s > cur_end:
            out.append((s - cur_end, prev, n))
        if e > cur_end:
            cur_end, prev = e, n
    tot = sum(g[0] for g in out)
    big = [g for g in out if g[0] >= 5000]
    print(f"last step: {len(out)} idle gaps, {tot / 1e3:.1f} us total; {len(big)} gaps >= 5 us "
          f"({sum(g[0] for g in big) / 1e3:.1f} us)")
    for g in sorted(out, reverse=True)[:top]:
        print(f"  {g[0] / 1e3:7.2f} us  {family(g[1])[:45]} -> {family(g[2])[:45]}")


if __name__ == "__main__":
    main()
