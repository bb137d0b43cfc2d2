"""GPU parity of the function-style gloo_amd.allreduce(AllreduceOptions)
(gloo/allreduce.cc:97-146; ring, bcube and the ring's all-links schedule)
through the C ABI glx_allreduce, against the reference's own outputs
(tests/golden/allreduce_fn_golden.*) and the oracle.  Thread-ranks sharing
one GPU and a HashStore, like gloo/test/allreduce_test.cc:306-356.
Bit-exact for every dtype."""
import os
import subprocess
import sys
import tempfile
import time

import numpy as np
import pytest

from helpers import (case_inputs, check_against_golden, fn_case_buffers,
                     load_allreduce_fn_golden, rank_env, run_ranks, same_bits)
from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from test_reduce_gpu import from_dev, to_dev  # noqa: E402

RING, BCUBE, RING_MESH = 1, 2, 3
INDEX, DATA = load_allreduce_fn_golden()


def gpu_allreduce_fn(algo, op, dtype, ins, outs, max_seg=0, runs=1, tag=0,
                     stream=False, rebind=False, timeout_s=60):
    """One gloo_amd.allreduce call per rank thread (per run).  rebind=True
    hands every run freshly allocated buffers (the cached executor must not
    depend on the previous call's pointers).  Returns outputs per rank."""
    import gloo_amd
    P = len(outs)
    N = outs[0][0].size
    store = gloo_amd.rendezvous.HashStore()
    result = [None] * P

    def upload(r):
        di = [to_dev(x, dtype) for x in ins[r]]
        do = [to_dev(x, dtype) for x in outs[r]]
        return di, do

    def rank_fn(r):
        ctx = gloo_amd.rendezvous.Context(r, P, 0)
        ctx.setTimeout(timeout_s)
        ctx.connectFullMesh(store)
        di, do = upload(r)
        for k in range(runs):
            if k > 0:
                if rebind:
                    di, do = upload(r)
                else:
                    for b, x in zip(di + do, ins[r] + outs[r]):
                        b.copy_(to_dev(x, dtype))
            torch.cuda.synchronize()
            opts = gloo_amd.AllreduceOptions(ctx)
            opts.setAlgorithm(algo)
            if di:
                opts.setInputs([b.data_ptr() for b in di], N, dtype=dtype)
            opts.setOutputs([b.data_ptr() for b in do], N, dtype=dtype)
            opts.setReduceFunction(op)
            opts.setMaxSegmentSize(max_seg)
            opts.setTag(tag)
            if stream:
                s = torch.cuda.Stream()
                opts.setStream(s)
                gloo_amd.allreduce(opts)
                s.synchronize()
            else:
                gloo_amd.allreduce(opts)
        result[r] = [from_dev(b, dtype) for b in do]
        ctx.close()
        return True

    run_ranks(P, rank_fn, timeout=timeout_s + 60)
    return result


def oracle_fn(algo, op, dtype, ins, outs, max_seg=0):
    return O.allreduce_fn(BCUBE if algo == BCUBE else RING, op, dtype, ins, outs, max_seg)


def check_outs(got, exp):
    for r in range(len(exp)):
        for i in range(len(exp[r])):
            assert same_bits(got[r][i], exp[r][i]), "rank %d output %d" % (r, i)


@pytest.mark.parametrize("rec", INDEX, ids=[r["name"] for r in INDEX])
def test_allreduce_fn_vs_reference_golden(rec):
    ins, outs = fn_case_buffers(rec)
    got = gpu_allreduce_fn(rec["algo"], rec["op"], rec["dtype"], ins, outs,
                           rec["max_segment_size"])
    for r in range(rec["P"]):
        for i in range(rec["nout"]):
            check_against_golden(rec, DATA, got[r][i])


RING_GOLDEN = [r for r in INDEX if r["algo"] == RING and r["P"] > 1]


@pytest.mark.parametrize("rec", RING_GOLDEN, ids=[r["name"] for r in RING_GOLDEN])
def test_ring_mesh_schedule_vs_reference_ring_golden(rec):
    ins, outs = fn_case_buffers(rec)
    got = gpu_allreduce_fn(RING_MESH, rec["op"], rec["dtype"], ins, outs,
                           rec["max_segment_size"])
    for r in range(rec["P"]):
        for i in range(rec["nout"]):
            check_against_golden(rec, DATA, got[r][i])


@pytest.mark.parametrize("algo", [RING, BCUBE, RING_MESH], ids=["ring", "bcube", "mesh"])
@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_large_buffers_vs_oracle(algo, P, monkeypatch):
    """(4 MiB + 3 elements) fp32 with 64 KiB segments and 256 KiB device
    pieces: many pieces per chunk, a ragged last one."""
    monkeypatch.setenv("GLOO_AMD_MIN_PIECE_BYTES", str(256 << 10))
    N = (1 << 20) + 3
    ins = [[] for _ in range(P)]
    outs = case_inputs(P, N, O.FLOAT32, 1, 0, seed=21)
    got = gpu_allreduce_fn(algo, O.SUM, O.FLOAT32, ins, outs, max_seg=64 << 10, runs=2)
    check_outs(got, oracle_fn(algo, O.SUM, O.FLOAT32, ins, outs, 64 << 10))


@pytest.mark.parametrize("algo", [RING, BCUBE, RING_MESH], ids=["ring", "bcube", "mesh"])
@pytest.mark.parametrize("dtype,op", [(O.FLOAT16, O.SUM), (O.BFLOAT16, O.SUM),
                                      (O.FLOAT16, O.MAX), (O.INT32, O.PRODUCT),
                                      (O.FLOAT64, O.MIN), (O.INT8, O.SUM)],
                         ids=lambda x: str(x))
def test_dtypes_inputs_outputs_rebind(algo, dtype, op):
    """Two inputs and two outputs per rank (seeded old outputs: float16's
    assignment reads them), new buffers on every call, user stream."""
    P, N = 5, 30011
    ins = case_inputs(P, N, dtype, 2, 0, seed=12)
    outs = [[O.fill(dtype, N, 0, seed=77, rank=r, ptr_index=i) for i in range(2)]
            for r in range(P)]
    got = gpu_allreduce_fn(algo, op, dtype, ins, outs, max_seg=4096, runs=3, rebind=True,
                           stream=True)
    if dtype == O.BFLOAT16:  # no reference type: the oracle's restatement
        exp = O.allreduce_fn(BCUBE if algo == BCUBE else RING, op, dtype, ins, outs, 4096)
    else:
        exp = oracle_fn(algo, op, dtype, ins, outs, 4096)
    check_outs(got, exp)


def test_distinct_tags_and_sizes_share_a_context():
    """Calls with different tags/sizes/algorithms interleave on one context;
    each keeps its own cached executor."""
    import gloo_amd
    P = 3
    store = gloo_amd.rendezvous.HashStore()
    cases = [(RING, 1000, 0), (BCUBE, 1000, 0), (RING, 1000, 7), (RING_MESH, 4099, 3),
             (RING, 1000, 0), (BCUBE, 77, 1)]
    data = {c: case_inputs(P, c[1], O.FLOAT32, 1, 0, seed=c[1] + c[2]) for c in cases}
    results = {}

    def rank_fn(r):
        ctx = gloo_amd.rendezvous.Context(r, P, 0)
        ctx.connectFullMesh(store)
        for rep in range(2):
            for c in cases:
                t = to_dev(data[c][r][0], O.FLOAT32)
                torch.cuda.synchronize()
                opts = gloo_amd.AllreduceOptions(ctx)
                opts.setAlgorithm(c[0])
                opts.setOutput(t)
                opts.setTag(c[2])
                opts.setReduceFunction(gloo_amd.ReductionFunction.sum)
                gloo_amd.allreduce(opts)
                results[(r, rep, c)] = from_dev(t, O.FLOAT32)
        ctx.close()
        return True

    run_ranks(P, rank_fn)
    for c in cases:
        exp = oracle_fn(c[0], O.SUM, O.FLOAT32, [[] for _ in range(P)], data[c])
        for r in range(P):
            for rep in range(2):
                assert same_bits(results[(r, rep, c)], exp[r][0]), (c, r, rep)


def test_timeout_raises_io_exception():
    """gloo/test/allreduce_test.cc:386-402: opts.setTimeout(10 ms) with a peer
    that never calls allreduce raises IoException("Timed out ...")."""
    import gloo_amd
    P = 2
    store = gloo_amd.rendezvous.HashStore()
    ctxs = [None, None]

    def rank_fn(r):
        ctxs[r] = gloo_amd.rendezvous.Context(r, P, 0)
        ctxs[r].connectFullMesh(store)
        return True

    run_ranks(P, rank_fn)
    buf = torch.ones(1, dtype=torch.float32, device="cuda")
    opts = gloo_amd.AllreduceOptions(ctxs[0])
    opts.setOutput(buf)
    opts.setReduceFunction(gloo_amd.math.sum)
    opts.setTimeout(0.01)
    t0 = time.time()
    with pytest.raises(gloo_amd.IoException, match="Timed out"):
        gloo_amd.allreduce(opts)
    assert time.time() - t0 < 5


def test_custom_reduce_function_needs_host_buffers():
    """A caller's function runs on the host (glx_allreduce_host_fn,
    tests/test_allreduce_custom.py): with device buffers allreduce() refuses
    it, naming why; something that is not a function is refused at once."""
    import torch

    import gloo_amd
    ctx = gloo_amd.rendezvous.Context(0, 1, 0)
    opts = gloo_amd.AllreduceOptions(ctx)
    with pytest.raises(gloo_amd.EnforceNotMet):
        opts.setReduceFunction("sum")
    opts.setReduceFunction(lambda c, a, b, n: None)
    opts.setOutput(torch.zeros(8, device="cuda"))
    with pytest.raises(gloo_amd.EnforceNotMet, match="host buffers"):
        gloo_amd.allreduce(opts)


WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mp_worker.py")


@pytest.mark.parametrize("algo", ["fn_ring", "fn_bcube", "fn_ring_mesh"])
def test_multiprocess_ipc(algo):
    P = 3
    with tempfile.TemporaryDirectory() as d:
        env = rank_env(P)
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P), algo],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(P)]
        outs = []
        for p in procs:
            try:
                o, _ = p.communicate(timeout=180)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs.append(o.decode(errors="replace"))
        for r, p in enumerate(procs):
            assert p.returncode == 0, "rank %d failed:\n%s" % (r, outs[r])
            assert "OK" in outs[r]


def host_allreduce_fn(algo, op, dtype, ins, outs, max_seg=0, runs=1):
    """gloo_amd.allreduce on host (numpy) buffers, the reference's calling
    convention; every call gets fresh arrays."""
    import gloo_amd
    P = len(outs)
    N = outs[0][0].size
    store = gloo_amd.rendezvous.HashStore()
    result = [None] * P

    def rank_fn(r):
        ctx = gloo_amd.rendezvous.Context(r, P, 0)
        ctx.setTimeout(60)
        ctx.connectFullMesh(store)
        for _ in range(runs):
            # the oracle keeps float16 as raw uint16 bits: hand numpy float16
            hv = np.float16 if dtype == O.FLOAT16 else None
            hi = [np.array(x, copy=True).view(hv) if hv else np.array(x, copy=True)
                  for x in ins[r]]
            ho = [np.array(x, copy=True).view(hv) if hv else np.array(x, copy=True)
                  for x in outs[r]]
            opts = gloo_amd.AllreduceOptions(ctx)
            opts.setAlgorithm(algo)
            if hi:
                opts.setInputs(hi, N)
            opts.setOutputs(ho, N)
            opts.setReduceFunction(op)
            opts.setMaxSegmentSize(max_seg)
            gloo_amd.allreduce(opts)
        result[r] = [x.view(np.uint16) for x in ho] if dtype == O.FLOAT16 else ho
        ctx.close()
        return True

    run_ranks(P, rank_fn, timeout=120)
    return result


HOST_GOLDEN = [r for r in INDEX if r["dtype"] != O.UINT64 or r["N"] in (0, 1000)]


@pytest.mark.parametrize("rec", HOST_GOLDEN, ids=[r["name"] for r in HOST_GOLDEN])
def test_allreduce_fn_host_buffers_vs_reference_golden(rec):
    ins, outs = fn_case_buffers(rec)
    got = host_allreduce_fn(rec["algo"], rec["op"], rec["dtype"], ins, outs,
                            rec["max_segment_size"], runs=2)
    for r in range(rec["P"]):
        for i in range(rec["nout"]):
            check_against_golden(rec, DATA, got[r][i])


@pytest.mark.parametrize("algo", [1, 2], ids=["ring", "bcube"])
@pytest.mark.parametrize("inplace", [True, False], ids=["in_place", "out_of_place"])
def test_allreduce_fn_host_staged_large(algo, inplace):
    """One host input (or in place) and one host output above the staging
    piece size: the overlapped path (H2D pieces in first-use order, each
    range copied back after its final write) -- same bits as the oracle."""
    P, N = 3, (5 << 20) + 3
    data = case_inputs(P, N, O.FLOAT32, 1, 0, seed=51)
    if inplace:
        ins, outs = [[] for _ in range(P)], data
    else:
        ins, outs = data, [[np.zeros(N, np.float32)] for _ in range(P)]
    got = host_allreduce_fn(algo, O.SUM, O.FLOAT32, ins, outs, runs=2)
    code = O.FN_BCUBE if algo == 2 else O.FN_RING
    exp = O.allreduce_fn(code, O.SUM, O.FLOAT32, [[] for _ in range(P)], data)
    for r in range(P):
        assert np.array_equal(got[r][0].view(np.uint32), exp[r][0].view(np.uint32)), r
