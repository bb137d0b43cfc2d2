"""HIP graph capture of the device-engine allreduce (tests/mp_worker.py
graph): one process per rank, each captures its algorithm's run() on its
stream with torch.cuda.graph and replays it with fresh inputs, mixed with
eager runs; every result exact, on every device engine (plan kernel: ring,
halving-doubling; two-shot: mesh; one-shot: replicated).  The kernels take
their run count / epoch from the device (kernels.h runCtr, epochCtr), so a
replay needs no host-side bookkeeping -- an MI355X-native way to put the
allreduce inside a captured training step."""
import os
import subprocess
import sys
import tempfile

import pytest

from helpers import rank_env

WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mp_worker.py")


@pytest.mark.gpu
@pytest.mark.parametrize("P", [2, 4])
def test_device_engine_graph_replays(P):
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P), "graph:40"],
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
    eng = [l for l in outs[0].splitlines() if l.startswith("ENGINES")][0]
    assert "'ring': 'devsteps'" in eng and "'hd': 'devsteps'" in eng, eng
    assert "'mesh': 'twoshot'" in eng and "'repl': 'oneshot'" in eng, eng


@pytest.mark.gpu
@pytest.mark.parametrize("kind,engine", [("ring", "devsteps"), ("mesh", "twoshot"),
                                         ("repl", "oneshot")])
def test_graph_replay_overlapping_an_eager_run_is_reported(kind, engine):
    """a replay on a stream that is not ordered after the
    algorithm's eager runs overlaps them; the device engine's launch counters
    detect it (xgmi_kernels.hip launch_number) and rank 0's next call raises
    EnforceNotMet instead of silently sharing a run number and landing slots.
    P = 2; rank 1 either completes or times out within 5 s."""
    P = 2
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P),
                                   "graph_overlap:" + kind],
                                  env=rank_env(P), stdout=subprocess.PIPE,
                                  stderr=subprocess.STDOUT) for r in range(P)]
        outs = []
        for p in procs:
            try:
                o, _ = p.communicate(timeout=120)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs.append(o.decode(errors="replace"))
    every = "\n".join("---- rank %d (rc %s) ----\n%s" % (r, p.returncode, outs[r][-2500:])
                       for r, p in enumerate(procs))
    assert procs[0].returncode == 0 and "VERDICT rank 0 overlap engine %s" % engine in outs[0], every
    assert procs[1].returncode == 0 and "OK" in outs[1], every


@pytest.mark.gpu
def test_freeing_after_a_reported_overlap_does_not_wait_out_the_timeout():
    """After an overlap stopped a launch early, its counters never settle:
    freeing the algorithm must see the device's report and return at once
    instead of draining until the context's 20 s timeout."""
    P = 2
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P),
                                   "graph_overlap:ring:close"],
                                  env=rank_env(P), stdout=subprocess.PIPE,
                                  stderr=subprocess.STDOUT) for r in range(P)]
        outs = []
        for p in procs:
            try:
                o, _ = p.communicate(timeout=120)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs.append(o.decode(errors="replace"))
    every = "\n".join("---- rank %d (rc %s) ----\n%s" % (r, p.returncode, outs[r][-2500:])
                       for r, p in enumerate(procs))
    assert all(p.returncode == 0 and "OK" in o for p, o in zip(procs, outs)), every
    assert "closed in" in outs[0], every
