"""gloo::allreduce(opts) with a caller's reduction function.

The reference's AllreduceOptions::Func (gloo/allreduce.h:36,69,171) may be
any host function.  On host buffers the product runs it on the host, in the
reference's order and operand order (glx_allreduce_host_fn, host_fn.cc).
Fixtures: tests/golden/allreduce_custom_golden.* -- the reference itself
(oracle/_ref) running gloo::allreduce with two custom Funcs over 32-bit
words: a bitwise or, and c = 3a + b mod 2^32 (neither commutative nor
associative: the bits pin every call's order and operands), RING and BCUBE,
P = 1..8, several inputs / outputs, segment sizes.

CPU: ranks as threads of this process (the function runs on the host; no GPU
is involved).  GPU suite: the same through one process per rank on the box
(the library as it ships there).
"""
import ctypes
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import threading

import numpy as np
import pytest

import gloo_amd
from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "allreduce_custom_golden")
with open(GOLDEN + ".json") as _f:
    CASES = json.load(_f)["cases"]
ARRAYS = np.load(GOLDEN + ".npz")
SEED = 1234
OR, THREE_A_PLUS_B = 100, 101


def words(addr, n):
    return np.frombuffer((ctypes.c_uint32 * n).from_address(addr), dtype=np.uint32)


def custom_fn(op):
    """The fixture's Func as a Python callable fn(c, a, b, n) on addresses."""
    def f_or(c, a, b, n):
        x, y = words(a, n).copy(), words(b, n).copy()
        words(c, n)[:] = x | y

    def f_3ab(c, a, b, n):
        x, y = words(a, n).copy(), words(b, n).copy()
        words(c, n)[:] = np.uint32(3) * x + y
    return {OR: f_or, THREE_A_PLUS_B: f_3ab}[op]


def buffers(c):
    """tests/golden/make_golden.py custom_case_buffers."""
    P, N = c["P"], c["N"]
    ins = [[O.fill(O.INT32, N, 0, seed=SEED + 7, rank=r, ptr_index=i) for i in range(c["nin"])]
           for r in range(P)]
    outs = [[O.fill(O.INT32, N, 0, seed=SEED + 8, rank=r, ptr_index=i)
             for i in range(c["nout"])] for r in range(P)]
    return ins, outs


def check_result(c, got):
    name = c["name"]
    if name in ARRAYS:
        return np.array_equal(got.view(np.uint32), ARRAYS[name].view(np.uint32))
    idx = ARRAYS[name + "_idx"]
    if not np.array_equal(got[idx].view(np.uint32), ARRAYS[name + "_sample"].view(np.uint32)):
        return False
    return hashlib.sha256(np.ascontiguousarray(got).tobytes()).hexdigest() == c["output_sha256"]


def run_rank(ctx, c, ins, outs):
    opts = gloo_amd.AllreduceOptions(ctx)
    opts.setAlgorithm(opts.Algorithm.BCUBE if c["algo"] == O.FN_BCUBE
                      else opts.Algorithm.RING)
    if ins:
        opts.setInputs(ins)
    opts.setOutputs(outs)
    opts.setReduceFunction(custom_fn(c["op"]))
    if c["max_segment_size"]:
        opts.setMaxSegmentSize(c["max_segment_size"])
    gloo_amd.allreduce(opts)


def thread_ranks(c):
    P = c["P"]
    ins, outs = buffers(c)
    store = gloo_amd.rendezvous.HashStore()
    errs = []

    def body(r):
        try:
            ctx = gloo_amd.rendezvous.Context(r, P)
            ctx.setTimeout(60)
            ctx.connectFullMesh(store)
            run_rank(ctx, c, ins[r], outs[r])
            ctx.close()
        except BaseException as e:  # noqa: BLE001
            errs.append((r, e))
    ts = [threading.Thread(target=body, args=(r,)) for r in range(P)]
    [t.start() for t in ts]
    [t.join(120) for t in ts]
    assert not errs, errs
    return outs


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_custom_function_matches_the_reference(case):
    outs = thread_ranks(case)
    for r in range(case["P"]):
        for i in range(case["nout"]):
            assert check_result(case, outs[r][i]), "rank %d output %d" % (r, i)


def test_custom_function_on_device_buffers_is_refused():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU: device buffers cannot be made")
    ctx = gloo_amd.rendezvous.Context(0, 1)
    t = torch.zeros(16, dtype=torch.int32, device="cuda")
    opts = gloo_amd.AllreduceOptions(ctx)
    opts.setOutputs([t])
    opts.setReduceFunction(custom_fn(OR))
    with pytest.raises(gloo_amd.EnforceNotMet, match="host buffers"):
        gloo_amd.allreduce(opts)


def test_custom_function_exception_propagates():
    """A Python reduction function that raises: the call fails with that
    exception (after the schedule ran), on every rank."""
    c = dict(CASES[0])
    c.update(P=1, N=8, nin=0, nout=2, max_segment_size=0)

    def boom(cc, a, b, n):
        raise ValueError("boom")
    ctx = gloo_amd.rendezvous.Context(0, 1)
    outs = [np.zeros(8, np.int32), np.ones(8, np.int32)]
    opts = gloo_amd.AllreduceOptions(ctx)
    opts.setOutputs(outs)
    opts.setReduceFunction(boom)
    with pytest.raises(ValueError, match="boom"):
        gloo_amd.allreduce(opts)


def test_a_failing_function_stops_the_call_and_its_peers_time_out():
    """Rank 0's function raises on its first call: rank 0's allreduce stops
    there and raises that exception; rank 1, whose function is fine, gets
    no result built from rank 0's unreduced data -- it waits for a message
    that never comes and raises IoException ("Timed out ..."), as the
    reference's ranks do when one rank's Func throws."""
    P = 2
    store = gloo_amd.rendezvous.HashStore()
    got = [None] * P

    def body(r):
        def fn(c, a, b, n):
            if r == 0:
                raise ValueError("rank 0 fails")
            custom_fn(OR)(c, a, b, n)
        try:
            ctx = gloo_amd.rendezvous.Context(r, P)
            ctx.setTimeout(2)
            ctx.connectFullMesh(store)
            opts = gloo_amd.AllreduceOptions(ctx)
            opts.setOutputs([np.arange(4096, dtype=np.int32)])
            opts.setReduceFunction(fn)
            gloo_amd.allreduce(opts)
            got[r] = "returned"
        except BaseException as e:  # noqa: BLE001
            got[r] = e
    ts = [threading.Thread(target=body, args=(r,)) for r in range(P)]
    [t.start() for t in ts]
    [t.join(60) for t in ts]
    assert isinstance(got[0], ValueError) and "rank 0 fails" in str(got[0]), got
    assert isinstance(got[1], gloo_amd.IoException) and "Timed out" in str(got[1]), got


@pytest.mark.parametrize("P", [3, pytest.param(2, marks=pytest.mark.gpu),
                               pytest.param(4, marks=pytest.mark.gpu)])
def test_custom_function_one_process_per_rank(P):
    """The fixtures' cases at P, one process per rank (mp_worker.py custom):
    the function runs on the host, so P = 3 runs in the CPU suite as well;
    the GPU suite runs P = 2 and 4 on the box."""
    worker = os.path.join(HERE, "mp_worker.py")
    with tempfile.TemporaryDirectory() as d:
        from helpers import rank_env
        procs = [subprocess.Popen([sys.executable, worker, d, str(r), str(P), "custom"],
                                  env=rank_env(P), stdout=subprocess.PIPE,
                                  stderr=subprocess.STDOUT) for r in range(P)]
        outs = []
        for p in procs:
            try:
                o, _ = p.communicate(timeout=300)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs.append(o.decode(errors="replace"))
        for r, p in enumerate(procs):
            assert p.returncode == 0 and "OK" in outs[r], "rank %d:\n%s" % (r, outs[r][-3000:])
