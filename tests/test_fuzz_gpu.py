"""GPU: randomized shapes (hypothesis, fixed seed, bounded example counts)
against the oracle, bit for bit -- off the parametrized grids:

* the reduce kernel (glx_reduce, gloo/math.h:15-73) with random lengths,
  element offsets of a, b and c chosen independently (so the three streams
  share a 16-byte phase, or do not and take the scalar path), in place or
  into a third buffer;
* the class allreduce on thread-ranks (host-issued steps: ranks sharing the
  box's one GPU) with random rank counts, lengths, pointer counts, dtypes,
  ops and schedules."""
import numpy as np
import pytest

hyp = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, seed, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

from helpers import case_inputs, same_bits  # noqa: E402
from oracle import oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from test_allreduce_gpu import MESH, gpu_allreduce  # noqa: E402
from test_reduce_gpu import ALL_DTYPES, ALL_OPS, assert_same, from_dev, to_dev  # noqa: E402

SETTINGS = dict(deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])


@settings(max_examples=600, **SETTINGS)
@seed(31)
@given(dtype=st.sampled_from(ALL_DTYPES), op=st.sampled_from(ALL_OPS),
       n=st.one_of(st.integers(1, 40), st.integers(41, 300000)),
       offs=st.tuples(st.integers(0, 17), st.integers(0, 17), st.integers(0, 17)),
       inplace=st.booleans())
def test_reduce_kernel_random_offsets(dtype, op, n, offs, inplace):
    import ctypes
    import gloo_amd
    from gloo_amd import _lib
    es = np.dtype(O.NP_DTYPE[dtype]).itemsize
    a = O.fill(dtype, n, 0, seed=n, rank=0)
    b = O.fill(dtype, n, 0, seed=n, rank=1)
    c0 = O.fill(dtype, n, 0, seed=n, rank=2)
    oa, ob, oc = offs
    if inplace:
        oc = oa
    pad = 32
    bufs = {}
    for key, x, o in (("a", a, oa), ("b", b, ob), ("c", c0, oc)):
        bufs[key] = to_dev(np.concatenate([np.zeros(o, x.dtype), x, np.zeros(pad, x.dtype)]),
                           dtype)
    pa = bufs["a"].data_ptr() + oa * es
    pb = bufs["b"].data_ptr() + ob * es
    C = bufs["a"] if inplace else bufs["c"]
    pc = C.data_ptr() + oc * es
    rc = _lib.lib.glx_reduce(op, dtype, ctypes.c_void_p(pc), ctypes.c_void_p(pa),
                             ctypes.c_void_p(pb), n,
                             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    gloo_amd.errors.check(rc, "glx_reduce")
    torch.cuda.synchronize()
    full = from_dev(C, dtype)
    assert np.all(full[:oc] == 0) and np.all(full[oc + n:] == 0), "wrote outside [c, c+n)"
    exp = O.reduce(op, dtype, a, b) if inplace else O.reduce(op, dtype, a, b, inplace=False, c=c0)
    assert_same(full[oc:oc + n], exp, dtype, op)


ALGOS = [O.RING_CHUNKED, O.HALVING_DOUBLING, MESH]


@settings(max_examples=200, **SETTINGS)
@seed(32)
@given(algo=st.sampled_from(ALGOS), P=st.integers(1, 9),
       N=st.one_of(st.integers(0, 64), st.integers(65, 200000)), nptrs=st.integers(1, 3),
       dtype=st.sampled_from([O.FLOAT32, O.FLOAT16, O.BFLOAT16, O.INT32, O.FLOAT64]),
       op=st.sampled_from(ALL_OPS))
def test_allreduce_random_shapes(algo, P, N, nptrs, dtype, op):
    ins = case_inputs(P, N, dtype, nptrs, 0, seed=P * 7 + N % 13)
    out = gpu_allreduce(algo, op, dtype, ins, runs=2)
    ref_algo = O.HALVING_DOUBLING if algo == O.HALVING_DOUBLING else O.RING_CHUNKED
    exp = O.allreduce(ref_algo, op, dtype, ins)
    for r in range(P):
        for i in range(nptrs):
            assert same_bits(out[r][i], exp[r][i]), (r, i)


@pytest.mark.parametrize("P,seed_", [(2, 1), (3, 2), (4, 3), (8, 4)])
def test_device_engines_random_cases_multiprocess(P, seed_):
    """One process per rank (the node's topology; the device engines run):
    100 random (algorithm, schedule, length, dtype, op, host/device buffer)
    cases per P, every rank against the oracle (mp_worker.py fuzz)."""
    import os
    import subprocess
    import sys
    import tempfile

    from helpers import rank_env
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mp_worker.py")
    with tempfile.TemporaryDirectory() as d:
        env = rank_env(P)
        procs = [subprocess.Popen([sys.executable, worker, d, str(r), str(P), "fuzz:%d" % seed_],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(P)]
        outs = []
        for p in procs:
            try:
                o, _ = p.communicate(timeout=420)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs.append(o.decode(errors="replace"))
        every = "\n".join("---- rank %d (rc %s) ----\n%s" % (r, p.returncode, outs[r][-3000:])
                          for r, p in enumerate(procs))
        print(outs[0][-2000:])
        for r, p in enumerate(procs):
            assert p.returncode == 0 and "OK" in outs[r], "rank %d failed:\n%s" % (r, every)
        # the DMA steps engine took part (about a third of the step-schedule cases)
        eng = [line for line in outs[0].splitlines() if line.startswith("ENGINES")][-1]
        assert "'dmasteps'" in eng, eng


SPLIT_ENVS = {
    # messages split at 64 KiB (GLOO_AMD_MAX_MESSAGE_BYTES, plan.cc
    # splitMessages): each piece its own channel and sub-region
    "split": {"GLOO_AMD_MAX_MESSAGE_BYTES": str(64 << 10)},
    # pipelined at 16 KiB (GLOO_AMD_PIPELINE_BYTES): the
    # host-issued and DMA steps forward every piece of a chunk on its own
    "pipelined": {"GLOO_AMD_PIPELINE_BYTES": str(16 << 10)},
}


@pytest.mark.parametrize("variant", sorted(SPLIT_ENVS))
@pytest.mark.parametrize("P,seed_", [(2, 5), (4, 6)])
def test_device_engines_random_cases_with_split_messages(P, seed_, variant):
    """The multi-process fuzz on split programs: the plan kernel, the
    host-issued and DMA steps (pipelined: the steps engines only), every rank
    bit for bit against the oracle."""
    import os
    import subprocess
    import sys
    import tempfile

    from helpers import rank_env
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mp_worker.py")
    with tempfile.TemporaryDirectory() as d:
        env = rank_env(P)
        env.update(SPLIT_ENVS[variant])
        env["FUZZ_CASES"] = "60"
        procs = [subprocess.Popen([sys.executable, worker, d, str(r), str(P), "fuzz:%d" % seed_],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(P)]
        outs = []
        for p in procs:
            try:
                o, _ = p.communicate(timeout=420)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs.append(o.decode(errors="replace"))
        every = "\n".join("---- rank %d (rc %s) ----\n%s" % (r, p.returncode, outs[r][-3000:])
                          for r, p in enumerate(procs))
        for r, p in enumerate(procs):
            assert p.returncode == 0 and "OK" in outs[r], "rank %d failed:\n%s" % (r, every)
        eng = [line for line in outs[0].splitlines() if line.startswith("ENGINES")][-1]
        assert "'devsteps'" in eng and "'dmasteps'" in eng, eng
