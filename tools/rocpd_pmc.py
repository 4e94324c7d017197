#!/usr/bin/env python3
"""Per-kernel mean PMC counter values from a rocprofv3 --pmc run's rocpd database (the default
output format): python tools/rocpd_pmc.py run_results.db [kernel-substring].  Prints each
counter's mean per dispatch and, with SQ_WAVE_CYCLES present, the wait / active fractions."""
import collections
import sqlite3
import sys


def main(db, pat=""):
    c = sqlite3.connect(db)
    rows = c.execute("select name, dispatch_id, counter_name, counter_value, duration from pmc_events").fetchall()
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    dur = collections.defaultdict(dict)
    for name, did, cn, cv, d in rows:
        if pat and pat not in name:
            continue
        per[name[:70]][did][cn] = per[name[:70]][did].get(cn, 0.0) + float(cv)
        dur[name[:70]][did] = d
    for k, ds in per.items():
        n = len(ds)
        tot = collections.Counter()
        for v in ds.values():
            tot.update(v)
        mean = {cn: v / n for cn, v in tot.items()}
        print(f"{k}  (dispatches {n}, mean duration {sum(dur[k].values()) / n / 1e3:.1f} us)")
        print("   " + "  ".join(f"{cn}={v:.4g}" for cn, v in sorted(mean.items())))
        wc = mean.get("SQ_WAVE_CYCLES")
        if wc:
            fr = {cn: mean[cn] / wc for cn in mean if cn != "SQ_WAVE_CYCLES" and ("WAIT" in cn or "ACTIVE" in cn or "BUSY" in cn)}
            print("   per wave-cycle: " + "  ".join(f"{cn[3:]}={v:.3f}" for cn, v in fr.items()))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
