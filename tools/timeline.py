#!/usr/bin/env python3
"""GPU timeline of one rank from a rocprofv3 --kernel-trace
[--memory-copy-trace] run (csv): every kernel and copy in start order with
its duration and the gap since the previous item ended, for the window of
the last `--last-us` microseconds (default: the last 3 ms).

    python tools/timeline.py PROFDIR/rank0 [--last-us 3000]
"""
import argparse
import csv
import os


def short(name):
    name = name.replace("(anonymous namespace)::", "").split("(")[0]
    for k in ("reduce_kernel", "copy_kernel", "reduce_n_kernel", "plan_kernel", "twoshot_kernel",
              "oneshot_kernel", "flag_ops_kernel", "copyBuffer", "elementwise_kernel", "fill"):
        if k in name:
            return k
    return name[-40:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix", help="PROFDIR/NAME (NAME_kernel_trace.csv etc.)")
    ap.add_argument("--last-us", type=float, default=3000.0)
    a = ap.parse_args()
    ev = []
    kt = a.prefix + "_kernel_trace.csv"
    for r in csv.DictReader(open(kt)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K q%s" % r.get("Queue_Id", "?"),
                   short(r["Kernel_Name"])))
    mt = a.prefix + "_memory_copy_trace.csv"
    if os.path.exists(mt):
        for r in csv.DictReader(open(mt)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C s%s" % r["Stream_Id"],
                       r["Direction"].replace("MEMORY_COPY_", "")))
    ev.sort()
    end = max(e[1] for e in ev)
    lo = end - a.last_us * 1e3
    win = [e for e in ev if e[1] >= lo]
    t0 = win[0][0]
    prev_end = None
    busy_end = t0
    for s, e, kind, name in win:
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        print("%9.1f  %8.1f us  gap %8.1f  %-8s %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, kind, name))
        prev_end = e if prev_end is None else max(prev_end, e)
        busy_end = max(busy_end, e)


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
