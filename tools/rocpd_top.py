#!/usr/bin/env python3
"""Per-kernel totals of a rocprofv3 rocpd database (count, mean us, total us), largest first,
and the last N dispatches with the gap before each: python tools/rocpd_top.py DB [--tail N]"""
import argparse
import collections
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--tail", type=int, default=12)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
    agg = collections.defaultdict(lambda: [0, 0.0])
    for n, s, e, *_ in rows:
        k = re.sub(r"\(.*", "", n).removeprefix("void ")[:70]
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1e3
    print(f"{len(rows)} dispatches")
    for k, (cnt, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"{cnt:6d} {t / cnt:9.2f} us {t:10.1f} us  {k}")
    print("--- last dispatches: us, grid, wg, gap before (us)")
    for i in range(max(1, len(rows) - a.tail), len(rows)):
        n, s, e, g, w = rows[i]
        print(f"{(e - s) / 1e3:8.2f} {g:8d} {w:5d} {(s - rows[i - 1][2]) / 1e3:8.2f}  {re.sub(r'[(].*', '', n)[:60]}")


if __name__ == "__main__":
    main()
