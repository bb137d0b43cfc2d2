#!/usr/bin/env python3
"""Run tests/mp_worker.py as P processes (one rank each) and fail unless every
rank prints OK -- the multi-process device-engine checks at a P the pytest
parametrisation does not cover (e.g. P=8 sharing one GPU).

    python tools/mp_workers.py P MODE [LOGDIR]
"""
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(os.path.dirname(HERE), "tests", "mp_worker.py")


def main():
    P, mode = int(sys.argv[1]), sys.argv[2]
    logdir = sys.argv[3] if len(sys.argv) > 3 else None
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P), mode], env=env,
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(P)]
        outs = [p.communicate()[0].decode(errors="replace") for p in procs]
    bad = 0
    for r, (p, o) in enumerate(zip(procs, outs)):
        if logdir:
            with open(os.path.join(logdir, "w%d_%s_r%d.log" % (P, mode, r)), "w") as f:
                f.write(o)
        ok = p.returncode == 0 and "OK" in o
        bad += not ok
        print("rank %d %s rc=%d" % (r, "OK" if ok else "FAILED", p.returncode), flush=True)
        if not ok:
            print(o[-3000:])
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
