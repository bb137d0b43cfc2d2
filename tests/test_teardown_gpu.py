"""Rank threads that close without a barrier.

tools/hop_latency_threads.py died once with SIGSEGV: its rank
threads closed their algorithm and context right after the last run, and
Store / Context / Algorithm handles may also be destroyed by the garbage
collector from whatever thread runs it.  This runs that teardown shape in a
subprocess with faulthandler on (a crash prints every thread's stack):
rounds of P = 2, 4, 8 thread-ranks on the box's GPU, each running the ring
and then closing at once -- explicitly, or by dropping the handles to the
garbage collector."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("close", ["explicit", "gc"])
def test_thread_ranks_close_without_a_barrier(close):
    cmd = [sys.executable, "-X", "faulthandler", os.path.join(ROOT, "tools", "stress_threads.py"),
           "--rounds", "6", "--runs", "20", "--close", close]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280)
    out = p.stdout + p.stderr
    assert p.returncode == 0 and "OK" in p.stdout, "rc %d:\n%s" % (p.returncode, out[-4000:])
