"""Kernel timeline around the last launch of a kernel family in a rocprofv3 rocpd database:
`python tools/kernel_tail.py run_results.db PATTERN [BEFORE] [AFTER]` prints the BEFORE kernels up
to the last one whose name matches PATTERN (regex) and AFTER kernels past it, with each kernel's
duration and its gap to the previous kernel's end (device-side launch / dependency cost)."""
import re
import sqlite3
import sys


def main():
    db, pat = sys.argv[1], re.compile(sys.argv[2])
    before = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    after = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    names = [re.sub(r"\(.*", "", n).replace("void ", "")[:60] for n, _, _ in rows]
    last = max((i for i, n in enumerate(names) if pat.search(n)), default=None)
    if last is None:
        print("no kernel matches", sys.argv[2])
        return
    lo, hi = max(0, last - before + 1), min(len(rows), last + after + 1)
    prev, busy, gaps = None, 0.0, 0.0
    for i in range(lo, hi):
        s, e = rows[i][1], rows[i][2]
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f"{(e - s) / 1e3:9.2f} us  gap {gap:8.2f} us  {names[i]}")
        busy += (e - s) / 1e3
        gaps += max(gap, 0.0)
        prev = e
    print(f"   busy {busy:.1f} us, gaps {gaps:.1f} us over {hi - lo} kernels")


if __name__ == "__main__":
    main()
