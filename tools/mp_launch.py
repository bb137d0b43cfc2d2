#!/usr/bin/env python3
"""Start P ranks of a torch.distributed program on this node (one process
each, MASTER_ADDR=127.0.0.1), optionally with rank 0 under rocprofv3 -- a
stand-in for torchrun when one rank needs a profiler in front of it.  This
launcher never touches the GPU; every rank is its own child process.

    python tools/mp_launch.py --nproc 2 [--prof-dir D] -- bench.py --gpus 2 ...
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
            argv = ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv",
                    "-d", a.prof_dir, "-o", "rank0", "--"] + argv
        procs.append(subprocess.Popen(argv, env=env))
    rc = 0
    for p in procs:
        rc = rc or p.wait()
    sys.exit(rc)


if __name__ == "__main__":
    main()
