"""Summarise a rocprofv3 rocpd SQLite database (kernel-trace) into a per-kernel stats table:
calls, total ms, mean us, share.  Usage: python tools/rocpd_summary.py <results.db> [steps]"""
import sqlite3
import sys


def main(path, steps=None):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end - start) from kernels group by {name} "
                     f"order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows)
    print(f"{'kernel':90s} {'calls':>7s} {'total_ms':>9s} {'mean_us':>8s} {'share':>6s}" +
          (f" {'ms/step':>8s}" if steps else ""))
    for n, k, t in rows:
        short = (n[:87] + "...") if len(n) > 90 else n
        line = f"{short:90s} {k:7d} {t / 1e6:9.3f} {t / k / 1e3:8.2f} {100 * t / total:5.1f}%"
        if steps:
            line += f" {t / 1e6 / steps:8.3f}"
        print(line)
    print(f"TOTAL kernel time {total / 1e6:.3f} ms" + (f" ({total / 1e6 / steps:.3f} ms/step)" if steps else ""))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else None)
