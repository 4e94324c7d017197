"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv (one row per dispatch x counter)."""
import collections
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.Counter())
    dur = collections.defaultdict(list)
    for r in rows:
        k = r["Kernel_Name"][:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
    for k, d in agg.items():
        vals = {c: v / cnt[k][c] for c, v in d.items()}
        print(k)
        print("   " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))
        wc = vals.get("SQ_WAVE_CYCLES")
        if wc:
            parts = {c: vals[c] / wc for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY") if c in vals}
            print("   fractions of wave-cycles: " + "  ".join(f"{c[3:]}={v:.2f}" for c, v in parts.items()))


if __name__ == "__main__":
    main(sys.argv[1])
