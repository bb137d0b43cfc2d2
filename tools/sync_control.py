"""Positive controls for the device engines' flag sync.

Runs the soak worker (tests/mp_worker.py soak: one process per rank sharing
the box's GPU, every run's result checked exactly) under the product's narrow
sync and under each TEST-ONLY broken mode (kernels.h kSyncNoAcquire,
kSyncNoRelease, kSyncUnsafe; GLOO_AMD_SYNC=unsafe_*), at sizes where every
workgroup re-reads a few KB of landing slot its CU read two runs before
(L1-warm: the guide's near-certain stale case without an acquire) and at the
soak's default 4 MiB, and writes how many runs per engine came out wrong.
A check that cannot fail a deliberately broken hand-off certifies nothing.

    python tools/sync_control.py OUT.json [--runs 200] [--P 2,4] [--n 4096,65536]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import rank_env  # noqa: E402

WORKER = os.path.join(ROOT, "tests", "mp_worker.py")
MODES = ["narrow", "unsafe_noacquire", "unsafe_norelease", "unsafe_test", "unsafe_cached"]


def soak(P, runs, n, mode, uneven, timeout):
    env = rank_env(P)
    env["GLOO_AMD_SYNC"] = mode
    t0 = time.time()
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P),
                                   "soak:%d:%s:%d" % (runs, uneven, n)],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(P)]
        outs = []
        for p in procs:
            try:
                o, _ = p.communicate(timeout=timeout)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                o = b"TIMEOUT"
            outs.append(o.decode(errors="replace"))
    bad = {}
    for r, o in enumerate(outs):
        m = re.search(r"BADRUNS rank \d+ (\{.*?\}) of", o)
        counts = eval(m.group(1)) if m else None  # noqa: S307 - our own worker's dict literal
        bad[r] = counts
    eng = next((l for l in outs[0].splitlines() if l.startswith("ENGINES")), None)
    return {"P": P, "n": n, "runs": runs, "mode": mode, "uneven": uneven or None,
            "rc": [p.returncode for p in procs], "bad_runs_per_rank": bad, "engines": eng,
            "seconds": round(time.time() - t0, 1),
            "tail_rank0": outs[0][-600:] if any(p.returncode for p in procs) else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--runs", type=int, default=200)
    ap.add_argument("--P", default="2,4")
    ap.add_argument("--n", default="4096,65536,1048576")
    ap.add_argument("--modes", default=",".join(MODES))
    ap.add_argument("--uneven", default="delays")
    ap.add_argument("--timeout", type=int, default=150)
    a = ap.parse_args()
    res = []
    for P in [int(x) for x in a.P.split(",")]:
        for n in [int(x) for x in a.n.split(",")]:
            for mode in a.modes.split(","):
                r = soak(P, a.runs, n, mode, a.uneven, a.timeout)
                res.append(r)
                print(json.dumps({k: r[k] for k in ("P", "n", "mode", "rc", "bad_runs_per_rank",
                                                     "seconds")}), flush=True)
                with open(a.out, "w") as f:
                    json.dump(res, f, indent=1)
                if any(rc is None or rc < 0 for rc in r["rc"]):
                    sys.exit("a rank died by a signal: stopping (%s)" % r["rc"])


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
