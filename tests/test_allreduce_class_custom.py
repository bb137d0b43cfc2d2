"""The class algorithms with a CUSTOM ReductionFunction<T> on host buffers.

The reference's AllreduceRingChunked<T> / AllreduceHalvingDoubling<T> take any
ReductionFunction<T>, including ReductionFunction<T>(CUSTOM, fn) with a
caller's fn(T* x, const T* y, n): x = f(x, y) (gloo/algorithm.h:56,58-83).
A device cannot run such a function; on host buffers the product runs the
algorithm's own program on the host (glx_allreduce_create_host_fn,
host_fn.h), calling fn where the reference calls fn_->call
(allreduce_ring_chunked.h:89-99,141-157; allreduce_halving_doubling.h:
231-273).  Fixtures: tests/golden/allreduce_class_custom_golden.*, the
reference itself (oracle/_ref) with two CUSTOM functions over 32-bit words --
x | y, and x = 3x + y mod 2^32 (neither commutative nor associative: the bits
pin every call's order and operands) -- P = 1..8, one to three pointers,
ragged counts.

CPU: ranks as threads of this process, and one process per rank at P = 3;
the GPU suite runs P = 2 and 4 one process per rank on the box.
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
from gloo_amd.algorithms import ReductionFunction, ReductionType
from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "allreduce_class_custom_golden")
with open(GOLDEN + ".json") as _f:
    CASES = json.load(_f)["cases"]
ARRAYS = np.load(GOLDEN + ".npz")
SEED = 1234
OR, THREE_X_PLUS_Y = 100, 101


def words(addr, n):
    return np.frombuffer((ctypes.c_uint32 * n).from_address(addr), dtype=np.uint32)


def class_fn(op):
    """The fixture's CUSTOM ReductionFunction: fn(x, y, n), x = f(x, y)."""
    def f_or(x, y, n):
        words(x, n)[:] |= words(y, n)

    def f_3xy(x, y, n):
        xs = words(x, n)
        xs[:] = np.uint32(3) * xs + words(y, n)
    return ReductionFunction(ReductionType.CUSTOM, {OR: f_or, THREE_X_PLUS_Y: f_3xy}[op])


def buffers(c):
    """tests/golden/make_golden.py case_inputs(P, N, INT32, nptrs, 0)."""
    return [[O.fill(O.INT32, c["N"], 0, seed=SEED, rank=r, ptr_index=i)
             for i in range(c["nptrs"])] for r in range(c["P"])]


def check_result(c, got):
    name = c["name"]
    if name in ARRAYS:
        return np.array_equal(got.view(np.uint32), ARRAYS[name].view(np.uint32))
    idx = ARRAYS[name + "_idx"]
    if not np.array_equal(got[idx].view(np.uint32), ARRAYS[name + "_sample"].view(np.uint32)):
        return False
    return hashlib.sha256(np.ascontiguousarray(got).tobytes()).hexdigest() == c["output_sha256"]


def make_alg(ctx, c, bufs):
    cls = (gloo_amd.AllreduceRingChunked if c["algo"] == O.RING_CHUNKED
           else gloo_amd.AllreduceHalvingDoubling)
    return cls(ctx, bufs, fn=class_fn(c["op"]))


def thread_ranks(c, runs=1):
    P = c["P"]
    bufs = buffers(c)
    store = gloo_amd.rendezvous.HashStore()
    errs = []
    engines = []

    def body(r):
        try:
            ctx = gloo_amd.rendezvous.Context(r, P)
            ctx.setTimeout(60)
            if P > 1:
                ctx.connectFullMesh(store)
            alg = make_alg(ctx, c, bufs[r])
            engines.append(alg.engine())
            for k in range(runs):
                if k:
                    for i, x in enumerate(buffers(c)[r]):
                        bufs[r][i][:] = x
                alg.run()
            alg.close()
            ctx.close()
        except BaseException as e:  # noqa: BLE001
            errs.append((r, e))
    ts = [threading.Thread(target=body, args=(r,)) for r in range(P)]
    [t.start() for t in ts]
    [t.join(120) for t in ts]
    assert not errs, errs
    assert set(engines) == {"hostfn"}, engines
    return bufs


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_class_custom_function_matches_the_reference(case):
    bufs = thread_ranks(case)
    for r in range(case["P"]):
        for i in range(case["nptrs"]):
            assert check_result(case, bufs[r][i]), "rank %d pointer %d" % (r, i)


def test_class_custom_function_runs_again_and_again():
    """Several run()s of one instance, the inputs refilled between them:
    every run equals the reference's (the executor's counters carry over)."""
    c = next(x for x in CASES if x["name"] == "hd_P5_N1000_3a_plus_b_p2")
    bufs = thread_ranks(c, runs=3)
    for r in range(c["P"]):
        for i in range(c["nptrs"]):
            assert check_result(c, bufs[r][i])


def test_class_custom_algorithms_created_and_freed_on_one_context():
    """Churn on one context: each rank builds an algorithm, runs it, frees it
    at once (no barrier) and builds the next, 30 times, alternating schedules
    and sizes.  A freed executor's counter words go back to the context and
    the next algorithm gets them: every receiver's last credit must have
    landed first (HostFnExecutor's destructor), else a late credit corrupts
    the next algorithm's counts.  Every run equals the reference's bits
    (the fixtures' cases at P = 4)."""
    cases = [c for c in CASES if c["P"] == 4]
    P = 4
    store = gloo_amd.rendezvous.HashStore()
    errs, bad = [], []

    def body(r):
        try:
            ctx = gloo_amd.rendezvous.Context(r, P)
            ctx.setTimeout(60)
            ctx.connectFullMesh(store)
            for k in range(30):
                c = cases[(k * 7) % len(cases)]
                bufs = buffers(c)[r]
                alg = make_alg(ctx, c, bufs)
                alg.run()
                alg.close()
                if not all(check_result(c, b) for b in bufs):
                    bad.append((r, k, c["name"]))
            ctx.close()
        except BaseException as e:  # noqa: BLE001
            errs.append((r, e))
    ts = [threading.Thread(target=body, args=(r,)) for r in range(P)]
    [t.start() for t in ts]
    [t.join(300) for t in ts]
    assert not errs, errs
    assert not bad, bad[:5]


def test_class_custom_function_on_device_buffers_is_refused():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU: device buffers cannot be made")
    ctx = gloo_amd.rendezvous.Context(0, 1)
    t = torch.zeros(16, dtype=torch.int32, device="cuda")
    with pytest.raises(gloo_amd.EnforceNotMet, match="host buffers"):
        gloo_amd.AllreduceRingChunked(ctx, [t], fn=class_fn(OR))


def test_class_custom_function_refusals():
    """Other class algorithms, streams, and the host-staging calls a
    host-run algorithm does not have are refused with a message."""
    ctx = gloo_amd.rendezvous.Context(0, 1)
    x = np.zeros(8, np.int32)
    with pytest.raises(gloo_amd.EnforceNotMet, match="AllreduceRingChunked or"):
        gloo_amd.AllreduceRing(ctx, [x], fn=class_fn(OR))
    with pytest.raises(ValueError, match="no streams"):
        gloo_amd.AllreduceHalvingDoubling(ctx, [x], fn=class_fn(OR), streams=[0])
    with pytest.raises(TypeError):
        ReductionFunction(ReductionType.CUSTOM, None)
    opts = gloo_amd.AllreduceOptions(ctx)
    with pytest.raises(gloo_amd.EnforceNotMet, match="callable fn"):
        opts.setReduceFunction(class_fn(OR))  # the function style takes a Func
    alg = gloo_amd.AllreduceRingChunked(ctx, [x], fn=class_fn(OR))
    with pytest.raises(gloo_amd.EnforceNotMet, match="runs on the host"):
        alg.run_fed()
    assert alg.transport_stats()["bytes"] == 0
    alg.close()


def test_class_custom_function_exception_propagates():
    def boom(x, y, n):
        raise ValueError("boom")
    ctx = gloo_amd.rendezvous.Context(0, 1)
    alg = gloo_amd.AllreduceRingChunked(ctx, [np.zeros(8, np.int32), np.ones(8, np.int32)],
                                        fn=ReductionFunction(ReductionType.CUSTOM, boom))
    with pytest.raises(ValueError, match="boom"):
        alg.run()
    alg.close()


@pytest.mark.parametrize("P", [3, pytest.param(2, marks=pytest.mark.gpu),
                               pytest.param(4, marks=pytest.mark.gpu)])
def test_class_custom_function_one_process_per_rank(P):
    """The fixtures' cases at P, one process per rank (mp_worker.py
    class_custom): the function runs on the host, so P = 3 runs in the CPU
    suite; the GPU suite runs P = 2 and 4 on the box."""
    worker = os.path.join(HERE, "mp_worker.py")
    from helpers import rank_env
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, worker, d, str(r), str(P), "class_custom"],
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
