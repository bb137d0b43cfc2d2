"""Soak: one instance per device engine run hundreds of times back to back
with fresh inputs each run, one process per rank (tests/mp_worker.py soak) --
the shape of a training job, which the grid tests (a few runs per instance)
do not reach: the plan kernel's run counter and per-run message numbers, the
one- and two-shot kernels' epochs and double-buffered slots, across many
kernel boundaries -- and the host-issued and DMA steps engines' counters
across as many runs.  Every run is checked exactly (integer-valued
inputs)."""
import os
import subprocess
import sys
import tempfile

import pytest

from helpers import rank_env

WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mp_worker.py")


@pytest.mark.gpu
@pytest.mark.parametrize("P,runs,mode,engines", [
    (2, 1000, "", "shared"), (4, 600, "", "shared"), (8, 300, "", "shared"),
    (4, 300, ":uneven", "shared"), (8, 300, ":delays", "shared"),
    (8, 100, ":uneven", None)])
def test_device_engines_soak(P, runs, mode, engines):
    """The guide's condition for testing hand-offs, uneven load: ":delays",
    random start delays per rank and run; ":uneven", also a GEMM stream busy
    on rank 0's GPU beside the collective.  engines: the ranks' device-engine
    mode ("shared": the rehearsal's opt-in to the device engines on the
    shared GPU; None: the library's automatic choice).  (8, 100, ":uneven")
    under the automatic choice is the configuration of the round-4 timeouts
    (8 ranks, one hardware queue each, a GEMM ahead of rank 0's collective
    while the other ranks' device engines held the CUs, profiles/r9j_*,
    r9l_*): the library now keeps ranks sharing a GPU on host-issued steps,
    which hold no CUs while they wait."""
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P),
                                   "soak:%d%s" % (runs, mode)],
                                  env=rank_env(P, device_engines=engines), stdout=subprocess.PIPE,
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
    eng = [l for l in outs[0].splitlines() if l.startswith("ENGINES")][0]
    if engines == "shared":
        # one rank per process: the device engines ran (not a host-steps fallback)
        assert "devsteps" in eng and "twoshot" in eng and "oneshot" in eng, eng
    else:
        # the automatic choice for ranks sharing a GPU: host-issued steps only
        assert "devsteps" not in eng and "twoshot" not in eng and "oneshot" not in eng, eng
    assert "'ring_host': 'steps'" in eng, eng
    # the DMA steps engine in every mode (its flag waits hold one wave, so the
    # shared-GPU starvation cycle cannot form: the (8, 100, ":uneven")
    # automatic case runs it beside rank 0's GEMMs)
    assert "'ring_dma': 'dmasteps'" in eng and "'hd_dma': 'dmasteps'" in eng, eng
