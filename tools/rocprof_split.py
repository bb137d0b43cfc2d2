#!/usr/bin/env python3
"""Per-loop split of a kernel's launches in a `rocprofv3 --kernel-trace`
trace of `bench.py` (N = 1), so the rocprof figure that backs
roofline.achieved is the timed loop's own, not the --stats average over
every loop of the run (warm, cold, staged legs).

    python tools/rocprof_split.py TRACE.csv [--warmup 5] [--steps 100] [--kernel reduce_kernel]

The bench (round 5) launches the kernel max(warmup, 4) times untimed over
its 4 rotating buffer pairs, then `steps` timed over the same rotation (HBM
only: the headline), then the warm loop back to back over one pair (2
untimed, then min(steps, 10) timed), then one check launch and the
host-staged legs.  Only launches with the largest grid are counted (the
staged legs fold 8 MiB pieces with a smaller grid).
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--kernel", default="reduce_kernel<float, 1,")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    grid = max(int(r.get("Grid_Size") or r["Grid_Size_X"]) for r in rows)
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows
           if int(r.get("Grid_Size") or r["Grid_Size_X"]) == grid]
    avg = lambda xs: sum(xs) / len(xs) if xs else float("nan")  # noqa: E731
    w, s = max(a.warmup, 4), a.steps
    timed = dur[w:w + s]
    warm_n = min(s, 10)
    warm = dur[w + s + 2:w + s + 2 + warm_n]
    print("kernel %s..., grid %d: %d launches" % (a.kernel, grid, len(dur)))
    print("  timed loop, 4 rotating pairs (launches %d..%d): %d launches, avg %.1f ns"
          % (w + 1, w + s, len(timed), avg(timed)))
    print("  warm loop, one pair (launches %d..%d, after 2 untimed): %d launches, avg %.1f ns"
          % (w + s + 3, w + s + 2 + warm_n, len(warm), avg(warm)))
    print("  all launches of that grid (the --stats line mixes every loop): avg %.1f ns"
          % avg(dur))


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
