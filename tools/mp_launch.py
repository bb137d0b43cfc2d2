#!/usr/bin/env python3
"""Start P ranks of a torch.distributed program on this node (one process
each, MASTER_ADDR=127.0.0.1), optionally with rank 0 under rocprofv3 -- a
stand-in for torchrun when one rank needs a profiler in front of it.  This
launcher never touches the GPU; every rank is its own child process.

    python tools/mp_launch.py --nproc 2 [--prof-dir D] [--pmc COUNTER] -- bench.py --gpus 2 ...

--pmc runs rank 0 under `rocprofv3 --pmc COUNTER` (one counter group per
pass: FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950) instead of
the kernel trace; tools/pmc_traffic.py reads the two passes' directories.
On a box where the ranks share one GPU the TCC counters are device-wide, so
a dispatch of rank 0 also counts what the other ranks' kernels moved in the
same window (DESIGN.md 4 says how the per-rank figure is derived).
"""
import argparse
import os
import subprocess
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nproc", type=int, required=True)
    ap.add_argument("--port", type=int, default=29581)
    ap.add_argument("--prof-dir", default=None,
                    help="rank 0 runs under rocprofv3 --kernel-trace --stats, output here")
    ap.add_argument("--pmc", default=None,
                    help="with --prof-dir: rank 0 runs under rocprofv3 --pmc <this> instead")
    ap.add_argument("--prof-name", default="rank0", help="rocprofv3 -o name")
    ap.add_argument("--copies", action="store_true",
                    help="with --prof-dir (no --pmc): also --memory-copy-trace")
    ap.add_argument("--api", action="store_true",
                    help="with --prof-dir (no --pmc): also --hip-runtime-trace")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    procs = []
    for r in range(a.nproc):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.nproc),
                   LOCAL_WORLD_SIZE=str(a.nproc), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(a.port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        argv = [sys.executable] + cmd
        if r == 0 and a.prof_dir:
            what = ["--pmc"] + a.pmc.split(",") if a.pmc else ["--kernel-trace", "--stats"]
            if a.copies and not a.pmc:
                what.append("--memory-copy-trace")
            if a.api and not a.pmc:
                what.append("--hip-runtime-trace")
            argv = ["rocprofv3"] + what + ["--output-format", "csv",
                                           "-d", a.prof_dir, "-o", a.prof_name, "--"] + argv
        procs.append(subprocess.Popen(argv, env=env))
    rc = 0
    for p in procs:
        rc = rc or p.wait()
    sys.exit(rc)


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
