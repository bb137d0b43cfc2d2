#!/usr/bin/env python3
"""HBM traffic per launch of the reduce kernel from rocprofv3 PMC passes.

Two separate passes (FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2; they do not
fit one pass on gfx950 -- MI355X_MICROARCH.md 'rocprofv3 PMC slots'):

  rocprofv3 --pmc FETCH_SIZE --output-format csv -d D -o fetch -- python3 bench.py --kernel-only
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d D -o write -- python3 bench.py --kernel-only
  python tools/pmc_traffic.py D [workload [kernel-substring [ranks-sharing-the-GPU]]]

With ranks sharing one GPU (the P = 8 rehearsal of the plan / two-shot
kernels, tools/mp_launch.py --pmc) the counters are device-wide: rank 0's
dispatch window also holds the other ranks' traffic.  The schedules are
symmetric and every rank's kernel waits on its peers, so the per-rank
estimate is the window's bytes / ranks (recorded as such).

Correction (MI355X_MICROARCH.md 'HBM'): FETCH_SIZE reports exactly half of
the bytes of a wide coalesced streaming read on gfx950 -> doubled; WRITE_SIZE
is exact for 16-B-per-lane streaming stores.  Both are in KiB.
Writes profiles/pmc_traffic.json.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(d, prefix, counter, kernel_substr="reduce_kernel"):
    files = glob.glob(os.path.join(d, "**", prefix + "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_substr not in row.get("Kernel_Name", ""):
                    continue
                if row.get("Counter_Name") != counter:
                    continue
                key = row.get("Dispatch_Id") or row.get("Correlation_Id")
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit("no %s samples for %s in %s" % (counter, kernel_substr, files))
    v = sorted(vals.values())
    # median over dispatches: the timed launches outnumber any small probe
    # launches of the same kernel
    return v[len(v) // 2], len(v)


def main():
    d = sys.argv[1]
    workload = sys.argv[2] if len(sys.argv) > 2 else "local_reduce_sum_fp32_256MiB"
    kernel = sys.argv[3] if len(sys.argv) > 3 else "reduce_kernel"
    ranks = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    fetch_kib, nf = per_launch(d, "fetch", "FETCH_SIZE", kernel)
    write_kib, nw = per_launch(d, "write", "WRITE_SIZE", kernel)
    hbm = (2 * fetch_kib + write_kib) * 1024
    rec = {"hbm_bytes_per_launch": int(hbm / ranks), "kernel": kernel,
           "fetch_size_kib_raw": fetch_kib, "write_size_kib": write_kib,
           "fetch_correction": "x2 (gfx950 FETCH_SIZE counts 64 B per 128-B request)",
           "dispatches": {"fetch": nf, "write": nw}, "source_dir": d}
    if ranks > 1:
        rec["device_bytes_per_window"] = int(hbm)
        rec["ranks_sharing_gpu"] = ranks
        rec["per_rank_note"] = ("device-wide counters over rank 0's dispatch window / ranks "
                                "(symmetric schedule, every rank on the one GPU)")
    out = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    data = {}
    if os.path.exists(out):
        with open(out) as f:
            data = json.load(f)
    data[workload] = rec
    with open(out, "w") as f:
        json.dump(data, f, indent=1)
    print(json.dumps({workload: rec}))


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
