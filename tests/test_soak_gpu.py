"""Soak: one instance per device engine run hundreds of times back to back
with fresh inputs each run, one process per rank (tests/mp_worker.py soak) --
the shape of a training job, which the grid tests (a few runs per instance)
do not reach: the plan kernel's run counter and per-run message numbers, the
one- and two-shot kernels' epochs and double-buffered slots, across many
kernel boundaries.  Every run is checked exactly (integer-valued inputs)."""
import os
import subprocess
import sys
import tempfile

import pytest

from helpers import rank_env

WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mp_worker.py")


@pytest.mark.gpu
@pytest.mark.parametrize("P,runs,mode", [(2, 1000, ""), (4, 600, ""), (8, 300, ""),
                                         (4, 300, ":uneven"), (8, 300, ":delays")])
def test_device_engines_soak(P, runs, mode):
    """The guide's condition for testing hand-offs, uneven load: ":delays",
    random start delays per rank and run; ":uneven", also a GEMM stream busy
    on rank 0's GPU beside the collective -- only where each process has two
    hardware queues (with one, 8 ranks sharing the GPU, the GEMM ahead of
    the collective in rank 0's only queue and the other ranks' collectives
    holding the CUs wait on each other: a cycle only ranks sharing a GPU can
    form; profiles/r9j_*, r9l_*)."""
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P),
                                   "soak:%d%s" % (runs, mode)],
                                  env=rank_env(P), stdout=subprocess.PIPE,
                                  stderr=subprocess.STDOUT) for r in range(P)]
        outs = []
        for p in procs:
            try:
                o, _ = p.communicate(timeout=150)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs.append(o.decode(errors="replace"))
    failed = [(r, p.returncode, o) for r, (p, o) in enumerate(zip(procs, outs))
              if p.returncode != 0 or "OK" not in o]
    # every failing rank's output: the first to fail is often not rank 0
    assert not failed, "\n".join("rank %d rc=%d:\n%s" % (r, rc, o[-2500:]) for r, rc, o in failed)
    # one rank per process: the device engines ran (not a host-steps fallback)
    eng = [l for l in outs[0].splitlines() if l.startswith("ENGINES")][0]
    assert "devsteps" in eng and "twoshot" in eng and "oneshot" in eng, eng
    assert "'ring_host': 'steps'" in eng, eng
