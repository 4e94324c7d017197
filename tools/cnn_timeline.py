"""Per-phase kernel timeline of `bench.py --model cnn` from a rocprofv3 rocpd database: the last 32
launches of each CNN bench (bound fused step bf16, fp32, recipe path): kernel, duration, and the
gap to the previous kernel's end (device-side launch / dependency cost)."""
import re
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    names = [re.sub(r"\(.*", "", n).replace("void ", "")[:60] for n, _, _ in rows]
    # the recipe path is the part after the first gather_batch launch
    gi = next((i for i, n in enumerate(names) if n.startswith("gather_batch")), len(rows))
    for title, lo, hi in (("bound fused steps (before the recipe path)", max(0, gi - 40), gi),
                          ("recipe path (Trainer.fit, fixed loader)", len(rows) - 48, len(rows))):
        print(f"== {title}")
        prev = None
        tot, gaps = 0.0, 0.0
        for i in range(lo, hi):
            n, s, e = names[i], rows[i][1], rows[i][2]
            gap = (s - prev) / 1e3 if prev is not None else 0.0
            print(f"{(e - s) / 1e3:9.2f} us  gap {gap:8.2f} us  {n}")
            tot += (e - s) / 1e3
            gaps += max(gap, 0.0)
            prev = e
        print(f"   busy {tot:.1f} us, gaps {gaps:.1f} us over {hi - lo} kernels")


if __name__ == "__main__":
    main()
