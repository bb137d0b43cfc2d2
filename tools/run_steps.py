#!/usr/bin/env python3
"""Run GPU-session steps in order, each under its own time limit, logging to
gpurun_out/<name>.log.  A step that FAILS (exit 1, e.g. a test assertion)
does not stop the session; a step that faults, aborts, segfaults or times out
(124/134/137/139 or a signal) ends it -- nothing more touches the GPU.

    python tools/run_steps.py steps.txt
steps file: one step per line:  name|timeout_seconds|shell command
"""
import os
import subprocess
import sys
import time

FATAL = {124, 134, 137, 139}


def main():
    steps = []
    with open(sys.argv[1]) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            name, tmo, cmd = line.split("|", 2)
            steps.append((name, int(tmo), cmd))
    os.makedirs("gpurun_out", exist_ok=True)
    summary = []
    for name, tmo, cmd in steps:
        log = os.path.join("gpurun_out", name + ".log")
        t0 = time.time()
        with open(log, "w") as f:
            rc = subprocess.call(["timeout", "-k", "10", str(tmo), "bash", "-c", cmd],
                                 stdout=f, stderr=subprocess.STDOUT)
        line = "%-24s rc=%-4d %6.1fs" % (name, rc, time.time() - t0)
        print(line, flush=True)
        summary.append(line)
        with open(os.path.join("gpurun_out", "summary.txt"), "w") as f:
            f.write("\n".join(summary) + "\n")
        if rc in FATAL or rc < 0:
            print("fatal exit status -- stopping the session", flush=True)
            return 1
    return 0


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    sys.exit(main())
