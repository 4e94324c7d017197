"""Join a --pmc counter_collection.csv with the kernel_trace.csv of the same run: per kernel
name, mean duration, GRBM cycles / duration (effective clock), MFMA instructions and the
MFMA-busy fraction.  Usage: python tools/pmc_clock_summary.py <rocprofv3 output dir>"""
import collections
import csv
import glob
import os
import sys


def main(d):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(cc)):
        vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    durs = collections.defaultdict(list)
    if kt:
        for r in csv.DictReader(open(kt[0])):
            durs[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        ds = durs.get(k, [0.0])
        dur = sum(ds) / len(ds)
        line = f"{k[:70]:70s} n={len(next(iter(cs.values())))} dur_us={dur:.1f}"
        if dur > 0:
            line += f" GRBM_COUNT/us={m.get('GRBM_COUNT', 0) / dur:.0f} GUI/us={m.get('GRBM_GUI_ACTIVE', 0) / dur:.0f}"
        line += " " + " ".join(f"{c}={v:.4g}" for c, v in sorted(m.items()))
        print(line)


if __name__ == "__main__":
    main(sys.argv[1])
