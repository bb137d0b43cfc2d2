#!/usr/bin/env python3
"""Per-launch medians of every counter in rocprofv3 --pmc output directories.

    python tools/pmc_summary.py KERNEL_SUBSTRING DIR [DIR ...] > summary.json

Each DIR holds one pass (*counter_collection.csv); the result maps DIR (its
basename) -> {counter: median over the kernel's dispatches, "dispatches": n}.
The raw CSVs are large (one row per dispatch and counter); the committed
profiles keep these summaries (tools/pmc_plan_excess.sh, pmc_dram.sh,
pmc_polls.sh make the passes)."""
import csv
import glob
import json
import os
import sys


def summarize(d, kernel):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel not in row.get("Kernel_Name", ""):
                    continue
                key = row.get("Dispatch_Id") or row.get("Correlation_Id")
                c = row["Counter_Name"]
                per.setdefault(c, {})
                per[c][key] = per[c].get(key, 0.0) + float(row["Counter_Value"])
    out = {}
    for c, vals in sorted(per.items()):
        v = sorted(vals.values())
        out[c] = v[len(v) // 2]
        out["dispatches"] = len(v)
    return out


def main():
    kernel, dirs = sys.argv[1], sys.argv[2:]
    print(json.dumps({os.path.basename(d.rstrip("/")): summarize(d, kernel) for d in dirs},
                     indent=1, sort_keys=True))


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
