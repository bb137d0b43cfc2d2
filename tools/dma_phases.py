#!/usr/bin/env python3
"""Where a DMA-driven ring's rounds go, from one rank's rocprofv3 kernel and
memory-copy traces of tools/hop_latency.py (--engines host_steps,dma_steps;
tools/gpu_recipes.sh timeline): the trace is cut into its four phases (host-issued steps
and DMA steps with on-GPU hand-offs, at each of two sizes, in the tool's
order), and for each phase the median duration of the SDMA copies, reduce and
copy kernels and flag-op kernels, and -- for the DMA steps -- the median time
from a copy's end to the start of the next kernel on the copy stream's queue
(the flag kernel that announces it: the SDMA -> compute-queue dependency).

    python tools/dma_phases.py PROFDIR/NAME
"""
import csv
import statistics as st
import sys


def kind_of(name):
    n = name.replace("(anonymous namespace)::", "")
    if "flag_ops_kernel" in n:
        return "flag"
    if n.startswith("void glx::reduce") or "glx::reduce_kernel" in n:
        return "reduce"
    if "glx::copy_kernel" in n:
        return "copyk"
    return "other"


def main():
    prefix = sys.argv[1]
    ev = []
    for r in csv.DictReader(open(prefix + "_kernel_trace.csv")):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind_of(r["Kernel_Name"]),
                   r["Queue_Id"]))
    for r in csv.DictReader(open(prefix + "_memory_copy_trace.csv")):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "SDMA", None))
    ev.sort()
    flags = [i for i, e in enumerate(ev) if e[2] == "flag"]
    # the DMA-steps phase of the first size ends at the first long pause
    # between flag kernels (the next phase is host-issued steps)
    cut = next(a for a, b in zip(flags, flags[1:]) if ev[b][0] - ev[a][1] > 2e6)
    rest = ev[cut + 1:]
    first_rest_flag = next(i for i, e in enumerate(rest) if e[2] == "flag")
    phases = [("host-issued steps, size 1", ev[:flags[0]]),
              ("DMA steps, size 1", ev[flags[0]:cut + 1]),
              ("host-issued steps, size 2", rest[:first_rest_flag]),
              ("DMA steps, size 2", rest[first_rest_flag:])]
    for name, es in phases:
        parts = []
        for k in ("SDMA", "reduce", "copyk", "flag"):
            d = [(e - s) / 1e3 for s, e, kk, q in es if kk == k]
            if d:
                parts.append("%s n=%d median %.1f us" % (k, len(d), st.median(d)))
        line = "%-26s %s" % (name, "; ".join(parts))
        fq = {q for s, e, kk, q in es if kk == "flag"}
        wq = {q for s, e, kk, q in es if kk in ("reduce", "copyk")}
        copy_q = fq - wq  # flag kernels alone on the copy stream's queue
        if copy_q:
            lat = []
            for i, (s, e, kk, q) in enumerate(es):
                if kk != "SDMA":
                    continue
                nxt = next((x for x in es[i + 1:] if x[3] in copy_q and x[0] >= e), None)
                if nxt is not None:
                    lat.append((nxt[0] - e) / 1e3)
            if lat:
                line += "; copy end -> next copy-stream kernel median %.1f us (n=%d)" % (
                    st.median(lat), len(lat))
        print(line)


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
