"""GPU parity of the MI355X allreduce path (HipAllreduceRingChunked /
HipAllreduceHalvingDoubling through the C ABI) against the oracle and the
reference's own outputs.  Ranks are threads sharing one GPU and a HashStore,
the reference's test topology (gloo/test/base_test.h:91-166); the copies are
intra-device, everything else (schedule, credits, progress engine) is the
multi-GPU code path.  Bit-exact for every dtype."""
import os
import subprocess
import sys
import tempfile
import time

import numpy as np
import pytest

from helpers import case_inputs, check_against_golden, load_allreduce_golden, rank_env, run_ranks
from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from test_reduce_gpu import TORCH_VIEW, assert_same, from_dev, to_dev  # noqa: E402

ALGOS = {O.RING_CHUNKED: "AllreduceRingChunked", O.HALVING_DOUBLING: "AllreduceHalvingDoubling",
         O.RING: "AllreduceRing", O.BCUBE: "AllreduceBcube"}


MESH = 2  # ring_chunked semantics, mesh schedule
REPL = 6  # ring_chunked semantics, one-round replicated schedule
AUTO = 8  # ring_chunked semantics, schedule chosen by size


def gpu_allreduce(algo, op, dtype, inputs, runs=1, streams=False, timeout_s=60,
                  refill_between_runs=True, base=2):
    """Run one algorithm instance per rank thread; returns results per rank/ptr."""
    import gloo_amd
    P, nptrs = len(inputs), len(inputs[0])
    N = inputs[0][0].size
    store = gloo_amd.rendezvous.HashStore()
    bufs = [[to_dev(x, dtype) for x in row] for row in inputs]
    torch.cuda.synchronize()
    fn = {O.SUM: gloo_amd.ReductionFunction.sum, O.PRODUCT: gloo_amd.ReductionFunction.product,
          O.MAX: gloo_amd.ReductionFunction.max, O.MIN: gloo_amd.ReductionFunction.min}[op]
    if algo in (MESH, REPL):
        def cls(*a, **kw):
            return gloo_amd.AllreduceRingChunked(
                *a, schedule="mesh" if algo == MESH else "replicated", **kw)
    elif algo == O.RING_CHUNKED:
        def cls(*a, **kw):
            return gloo_amd.AllreduceRingChunked(*a, schedule="ring", **kw)
    elif algo == AUTO:
        cls = gloo_amd.AllreduceRingChunked
    else:
        cls = getattr(gloo_amd, ALGOS[algo])

    def rank_fn(r):
        ctx = gloo_amd.rendezvous.Context(r, P, 0)
        ctx.setTimeout(timeout_s)
        ctx.connectFullMesh(store)
        ctx.base = base  # gloo::Context::base (AllreduceBcube's group size)
        ptrs = [b.data_ptr() for b in bufs[r]]
        ss = [torch.cuda.Stream() for _ in range(nptrs)] if streams else None
        alg = cls(ctx, ptrs, N, fn, streams=ss, dtype=dtype)
        for k in range(runs):
            if k > 0 and refill_between_runs:
                for i in range(nptrs):
                    bufs[r][i].copy_(to_dev(inputs[r][i], dtype))
                torch.cuda.synchronize()
            alg.run()
            if streams:
                ss[0].synchronize()
        alg.close()
        return True

    run_ranks(P, rank_fn, timeout=timeout_s + 30)
    torch.cuda.synchronize()
    return [[from_dev(b, dtype) for b in row] for row in bufs]


def check_all(out, exp, dtype, op):
    for r in range(len(exp)):
        for i in range(len(exp[r])):
            assert_same(out[r][i], exp[r][i], dtype, op)


@pytest.mark.parametrize("algo", [O.RING_CHUNKED, O.HALVING_DOUBLING],
                         ids=["ring_chunked", "halving_doubling"])
@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("N", [0, 1, 255, 256, 1000, 4099, 100003])
def test_allreduce_fp32_vs_oracle(algo, P, N):
    ins = case_inputs(P, N, O.FLOAT32, 1, 0)
    out = gpu_allreduce(algo, O.SUM, O.FLOAT32, ins)
    check_all(out, O.allreduce(algo, O.SUM, O.FLOAT32, ins), O.FLOAT32, O.SUM)


INDEX, DATA = load_allreduce_golden()


@pytest.mark.parametrize("rec", INDEX, ids=[r["name"] for r in INDEX])
def test_allreduce_vs_reference_golden(rec):
    ins = case_inputs(rec["P"], rec["N"], rec["dtype"], rec["nptrs"], rec["kind"], rec["seed"])
    out = gpu_allreduce(rec["algo"], rec["op"], rec["dtype"], ins)
    for r in range(rec["P"]):
        for i in range(rec["nptrs"]):
            check_against_golden(rec, DATA, out[r][i])


# The reference test suite's own grid (gloo/test/allreduce_test.cc:251-269):
# AllreduceRingChunked at P = 1..15 x N in {0, 4, 100, 1000, 10000} and
# AllreduceHalvingDoubling at P in {1..9, 13, 16, 24, 32} x N in {0, 1, 64,
# 1000}, SinglePointer (:143-169): rank r contributes value r, every element
# must equal P(P-1)/2 exactly.  Thread-ranks on one GPU, like the reference's
# ranks-as-threads tests (gloo/test/base_test.h:91-166).
REF_GRID = ([(O.RING_CHUNKED, P, N) for P in range(1, 16) for N in (0, 4, 100, 1000, 10000)] +
            [(O.HALVING_DOUBLING, P, N) for P in (1, 2, 3, 4, 5, 6, 7, 8, 9, 13, 16, 24, 32)
             for N in (0, 1, 64, 1000)])


@pytest.mark.parametrize("algo,P,N", REF_GRID,
                         ids=["%s-P%d-N%d" % ("ring_chunked" if a == O.RING_CHUNKED
                                              else "halving_doubling", P, N)
                              for a, P, N in REF_GRID])
def test_reference_test_grid_single_pointer(algo, P, N):
    ins = [[np.full(N, r, dtype=np.float32)] for r in range(P)]
    out = gpu_allreduce(algo, O.SUM, O.FLOAT32, ins, runs=2)
    for r in range(P):
        assert np.all(out[r][0] == P * (P - 1) // 2), "rank %d" % r


# The CUDA algorithms' test grid (gloo/test/cuda_allreduce_test.cc:148-170,
# 281-309: the same ranks, N without 0) with CudaFixture's values, the stride
# pattern (gloo/test/base_test.h:184-192) checked for exact equality
# (checkAllreduceResult, :216-236).
@pytest.mark.parametrize("algo,P,N", [g for g in REF_GRID if g[2] > 0],
                         ids=["%s-P%d-N%d" % ("ring_chunked" if a == O.RING_CHUNKED
                                              else "halving_doubling", P, N)
                              for a, P, N in REF_GRID if N > 0])
def test_cuda_test_grid_stride_pattern(algo, P, N):
    ins = case_inputs(P, N, O.FLOAT32, 1, 1)
    out = gpu_allreduce(algo, O.SUM, O.FLOAT32, ins)
    j = np.arange(N, dtype=np.float64)
    exp = (j * P * P + P * (P - 1) / 2).astype(np.float32)
    for r in range(P):
        assert np.array_equal(out[r][0], exp), "rank %d" % r


# Beyond 8 ranks with seeded inputs, so the reduction ORDER is checked too
# (value = rank sums exactly in any order): bit-exact against the oracle.
@pytest.mark.parametrize("algo,P", [(O.RING_CHUNKED, 11), (O.RING_CHUNKED, 15),
                                    (O.HALVING_DOUBLING, 13), (O.HALVING_DOUBLING, 16),
                                    (O.HALVING_DOUBLING, 24), (O.HALVING_DOUBLING, 32)],
                         ids=["ring_chunked-P11", "ring_chunked-P15", "halving_doubling-P13",
                              "halving_doubling-P16", "halving_doubling-P24",
                              "halving_doubling-P32"])
@pytest.mark.parametrize("N", [1000, 10007])
def test_many_ranks_vs_oracle(algo, P, N):
    ins = case_inputs(P, N, O.FLOAT32, 1, 0, seed=31)
    out = gpu_allreduce(algo, O.SUM, O.FLOAT32, ins)
    check_all(out, O.allreduce(algo, O.SUM, O.FLOAT32, ins), O.FLOAT32, O.SUM)


@pytest.mark.parametrize("algo", [O.RING_CHUNKED, O.HALVING_DOUBLING],
                         ids=["ring_chunked", "halving_doubling"])
@pytest.mark.parametrize("dtype", [O.INT8, O.INT32, O.INT64, O.UINT64, O.FLOAT64,
                                   O.FLOAT16, O.BFLOAT16],
                         ids=lambda d: O.DTYPE_NAMES[d])
@pytest.mark.parametrize("op", [O.SUM, O.PRODUCT, O.MAX, O.MIN],
                         ids=lambda o: O.OP_NAMES[o])
def test_allreduce_dtypes_ops(algo, dtype, op):
    P, N = 3, 3001
    ins = case_inputs(P, N, dtype, 1, 0, seed=77)
    out = gpu_allreduce(algo, op, dtype, ins)
    check_all(out, O.allreduce(algo, op, dtype, ins), dtype, op)


@pytest.mark.parametrize("algo", [O.RING_CHUNKED, O.HALVING_DOUBLING],
                         ids=["ring_chunked", "halving_doubling"])
def test_multi_pointer_and_repeated_runs(algo):
    """ptrs.size() > 1 (local fold + broadcast) and run() repeated on one
    instance (credits carry across runs, gloo/allreduce_ring_chunked.h:202-206)."""
    P, N, nptrs = 4, 20000, 3
    ins = case_inputs(P, N, O.FLOAT32, nptrs, 0, seed=9)
    out = gpu_allreduce(algo, O.SUM, O.FLOAT32, ins, runs=3)
    check_all(out, O.allreduce(algo, O.SUM, O.FLOAT32, ins), O.FLOAT32, O.SUM)


@pytest.mark.parametrize("algo", [O.RING_CHUNKED, O.HALVING_DOUBLING],
                         ids=["ring_chunked", "halving_doubling"])
def test_user_streams(algo):
    P, N = 4, 300000
    ins = case_inputs(P, N, O.FLOAT32, 1, 0, seed=21)
    out = gpu_allreduce(algo, O.SUM, O.FLOAT32, ins, runs=2, streams=True)
    check_all(out, O.allreduce(algo, O.SUM, O.FLOAT32, ins), O.FLOAT32, O.SUM)


@pytest.mark.parametrize("algo", [O.RING_CHUNKED, O.HALVING_DOUBLING, MESH],
                         ids=["ring_chunked", "halving_doubling", "mesh"])
@pytest.mark.parametrize("P,nptrs", [(1, 2), (2, 2), (3, 3), (4, 2)])
def test_multi_pointer_async_streams(algo, P, nptrs):
    """gloo/test/cuda_allreduce_test.cc:196-220 (MultiPointerAsync): one stream
    per pointer; each pointer's values are written on ITS stream behind a
    delay kernel (cudaSleep, gloo/test/cuda_base_test.h:60-74), nothing
    synchronises before run(), and the results are read after synchronising
    the streams (:216-218).  run() must order itself after every pointer's
    pending work and every stream's later work after the results.  The
    fixture's stride pattern (gloo/test/base_test.h:184-235) sums exactly."""
    import gloo_amd
    N = 3001
    store = gloo_amd.rendezvous.HashStore()
    stride = P * nptrs
    j = np.arange(N, dtype=np.float64)
    expected = (j * stride * stride + stride * (stride - 1) / 2).astype(np.float32)
    cls = {O.RING_CHUNKED: lambda *a, **k: gloo_amd.AllreduceRingChunked(*a, schedule="ring", **k),
           O.HALVING_DOUBLING: gloo_amd.AllreduceHalvingDoubling,
           MESH: lambda *a, **k: gloo_amd.AllreduceRingChunked(*a, schedule="mesh", **k)}[algo]

    def rank_fn(r):
        ctx = gloo_amd.rendezvous.Context(r, P, 0)
        ctx.setTimeout(60)
        ctx.connectFullMesh(store)
        ss = [torch.cuda.Stream() for _ in range(nptrs)]
        bufs = [torch.zeros(N, device="cuda") for _ in range(nptrs)]
        host = [torch.from_numpy((j * stride + r * nptrs + i).astype(np.float32)).pin_memory()
                for i in range(nptrs)]
        torch.cuda.synchronize()
        alg = cls(ctx, [b.data_ptr() for b in bufs], N, gloo_amd.ReductionFunction.sum,
                  streams=ss, dtype=O.FLOAT32)
        for _ in range(2):
            for i in range(nptrs):
                with torch.cuda.stream(ss[i]):
                    bufs[i].zero_()
                    torch.cuda._sleep(200000)  # the fixture's cudaSleep
                    bufs[i].copy_(host[i], non_blocking=True)
            alg.run()
            for st in ss:
                st.synchronize()
            for i in range(nptrs):
                got = bufs[i].cpu().numpy()
                assert np.array_equal(got, expected), "rank %d ptr %d" % (r, i)
        alg.close()
        return True

    run_ranks(P, rank_fn, timeout=90)


def test_streams_must_match_pointers():
    """CudaAllreduceRingChunked enforces one stream per pointer
    (gloo/cuda_allreduce_ring_chunked.cc:55-58); one stream is also taken."""
    import gloo_amd
    store = gloo_amd.rendezvous.HashStore()
    ctx = gloo_amd.rendezvous.Context(0, 1, 0)
    ctx.connectFullMesh(store)
    bufs = [torch.zeros(100, device="cuda") for _ in range(3)]
    ss = [torch.cuda.Stream() for _ in range(2)]
    with pytest.raises(gloo_amd.EnforceNotMet, match="one per pointer"):
        gloo_amd.AllreduceRingChunked(ctx, [b.data_ptr() for b in bufs], 100,
                                      gloo_amd.ReductionFunction.sum, streams=ss,
                                      dtype=O.FLOAT32)


def test_back_to_back_without_refill_is_iterated_allreduce():
    """Two runs without refilling = allreduce applied twice (the benchmark
    loop of gloo/benchmark/runner.cc:361-392)."""
    P, N = 4, 50000
    ins = case_inputs(P, N, O.INT32, 1, 0, seed=4)
    out = gpu_allreduce(O.RING_CHUNKED, O.SUM, O.INT32, ins, runs=2, refill_between_runs=False)
    once = O.allreduce(O.RING_CHUNKED, O.SUM, O.INT32, ins)
    twice = O.allreduce(O.RING_CHUNKED, O.SUM, O.INT32, once)
    check_all(out, twice, O.INT32, O.SUM)


def test_multiple_algorithms_one_context():
    """gloo/test/allreduce_test.cc:171-210: several algorithms on one context,
    each run twice (slots must not collide)."""
    import gloo_amd
    P, N = 4, 1000
    store = gloo_amd.rendezvous.HashStore()
    bufs = [torch.full((N,), float(r), device="cuda") for r in range(P)]
    torch.cuda.synchronize()

    def rank_fn(r):
        ctx = gloo_amd.rendezvous.Context(r, P, 0)
        ctx.connectFullMesh(store)
        algs = [gloo_amd.AllreduceRingChunked(ctx, [bufs[r]]),
                gloo_amd.AllreduceHalvingDoubling(ctx, [bufs[r]])]
        for alg in algs:
            for _ in range(2):
                bufs[r].fill_(float(r))
                torch.cuda.synchronize()
                alg.run()
                assert torch.all(bufs[r] == P * (P - 1) / 2).item()
        return True

    run_ranks(P, rank_fn)


def test_timeout_raises_io_exception():
    """gloo/test/allreduce_test.cc:386-402: a short timeout with a peer that
    never joins the collective raises IoException("Timed out ...")."""
    import gloo_amd
    P = 2
    store = gloo_amd.rendezvous.HashStore()
    buf = torch.ones(1024, device="cuda")
    ctxs = [None, None]

    def rank_fn(r):
        ctx = gloo_amd.rendezvous.Context(r, P, 0)
        ctx.connectFullMesh(store)
        ctxs[r] = ctx
        return ctx

    run_ranks(P, rank_fn)
    ctx = ctxs[0]
    ctx.setTimeout(0.05)
    alg = gloo_amd.AllreduceRingChunked(ctx, [buf])
    t0 = time.time()
    with pytest.raises(gloo_amd.IoException, match="Timed out"):
        alg.run()
    assert time.time() - t0 < 5


@pytest.mark.parametrize("P", [2, 3, 4, 8])
@pytest.mark.parametrize("N", [1, 255, 1000, 4099, 100003])
def test_mesh_schedule_matches_ring_chunked_oracle(P, N):
    ins = case_inputs(P, N, O.FLOAT32, 1, 0, seed=8)
    out = gpu_allreduce(MESH, O.SUM, O.FLOAT32, ins, runs=2)
    check_all(out, O.allreduce(O.RING_CHUNKED, O.SUM, O.FLOAT32, ins), O.FLOAT32, O.SUM)


@pytest.mark.parametrize("dtype,op", [(O.FLOAT32, O.MAX), (O.FLOAT16, O.SUM),
                                      (O.BFLOAT16, O.SUM), (O.INT32, O.PRODUCT),
                                      (O.FLOAT64, O.MIN)],
                         ids=lambda x: str(x))
def test_mesh_schedule_dtypes(dtype, op):
    P, N = 5, 30011
    ins = case_inputs(P, N, dtype, 2, 0, seed=12)
    out = gpu_allreduce(MESH, op, dtype, ins, streams=True)
    check_all(out, O.allreduce(O.RING_CHUNKED, op, dtype, ins), dtype, op)


RING_GOLDEN = [r for r in INDEX if r["algo"] == O.RING_CHUNKED]


@pytest.mark.parametrize("rec", RING_GOLDEN, ids=[r["name"] for r in RING_GOLDEN])
def test_mesh_schedule_vs_reference_ring_golden(rec):
    ins = case_inputs(rec["P"], rec["N"], rec["dtype"], rec["nptrs"], rec["kind"], rec["seed"])
    out = gpu_allreduce(MESH, rec["op"], rec["dtype"], ins)
    for r in range(rec["P"]):
        for i in range(rec["nptrs"]):
            check_against_golden(rec, DATA, out[r][i])


WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mp_worker.py")


@pytest.mark.parametrize("algo", ["ring_chunked", "halving_doubling", "ring_chunked_mesh"])
def test_multiprocess_ipc(algo):
    """One process per rank (the torchrun topology): endpoints via a FileStore,
    receive regions shared with hipIpcGetMemHandle/hipIpcOpenMemHandle."""
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


@pytest.mark.parametrize("P,mode", [(P, m) for P in (2, 3, 4)
                                    for m in ("oneshot", "twoshot", "devsteps", "dmasteps")] +
                         [(8, "devsteps"), (8, "dmasteps")])
def test_device_engine_multiprocess(P, mode):
    """The replicated (one-shot) and mesh (two-shot) schedules, and the ring,
    halving-doubling and bcube step programs (plan kernel), as one
    device-driven kernel per rank (xgmi_kernels.hip), one process per rank:
    peers' kernels push into each other's IPC-mapped uncached regions and
    wait on flags.  Bit-exact with the reference ring's chains for every
    dtype/op, device and host buffers, class and function style, repeated
    runs, ranges left empty at small sizes (mp_worker.py).  dmasteps: the
    same cases through the DMA steps engine (the host-issued program, its
    hand-offs made on the GPU by flag kernels)."""
    with tempfile.TemporaryDirectory() as d:
        env = rank_env(P)
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P), mode],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(P)]
        outs = []
        for p in procs:
            try:
                o, _ = p.communicate(timeout=420 if P > 4 else 240)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs.append(o.decode(errors="replace"))
        # every rank's output on a failure: a rank's own timeout report says
        # which step and flag it waited for, and only all of them together
        # show where a cycle of waits closed
        every = "\n".join("---- rank %d (rc %s) ----\n%s" % (r, p.returncode, outs[r])
                          for r, p in enumerate(procs))
        for r, p in enumerate(procs):
            assert p.returncode == 0 and "OK" in outs[r], "rank %d failed:\n%s" % (r, every)


@pytest.mark.parametrize("P,engine,when", [(2, "host", "idle"), (3, "host", "mid"),
                                           (3, "device", "idle"), (3, "device", "mid"),
                                           (3, "dma", "idle"), (3, "dma", "mid"),
                                           (3, "twoshot", "idle"), (3, "twoshot", "mid")])
def test_peer_killed_raises_io_exception(P, engine, when):
    """Fault injection as TransportMultiProcTest.IoErrors
    (gloo/test/transport_test.cc:53-110, P in {2,3,4}): rank 0 is SIGKILLed
    while idle or in the middle of its own run(); every survivor's run()
    raises IoException('Connection closed by peer') well within the 3 s
    timeout (the reference allows 2x): the host engine's loop and the device
    engines' host wait both watch the peers' processes, and on an exit the
    latter stop their kernels' waits through the status word.  Survivors
    then close cleanly."""
    with tempfile.TemporaryDirectory() as d:
        env = rank_env(P)
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P),
                                   "killpeer:%s:%s" % (engine, when)],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(P)]
        outs = [None] * P
        # survivors first: the killed rank stays an unreaped zombie meanwhile,
        # which the liveness check must still see as gone
        for r in list(range(1, P)) + [0]:
            p = procs[r]
            try:
                o, _ = p.communicate(timeout=120)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs[r] = o.decode(errors="replace")
        assert procs[0].returncode == -9, outs[0]
        for r in range(1, P):
            print(outs[r])
            assert procs[r].returncode == 0, "rank %d failed:\n%s" % (r, outs[r])
            assert "OK" in outs[r]


@pytest.mark.parametrize("mode,knob", [("devsteps", "GLOO_AMD_FLAG_WRITE=store"),
                                       ("dmasteps", "GLOO_AMD_FLAG_WRITE=store"),
                                       ("twoshot", "GLOO_AMD_FLAG_WRITE=store"),
                                       ("oneshot", "GLOO_AMD_FLAG_WRITE=store"),
                                       ("devsteps", "GLOO_AMD_FUSE=0"),
                                       ("devsteps", "GLOO_AMD_ENGINE_STREAMS=fast"),
                                       ("devsteps", "GLOO_AMD_SYNC=system"),
                                       ("twoshot", "GLOO_AMD_SYNC=system"),
                                       ("oneshot", "GLOO_AMD_SYNC=system")])
def test_device_engine_variants(mode, knob):
    """The device engines' other forms, same checks as above at P=3: flag
    words written with system-scope stores (what ranks use when the link to a
    peer's GPU carries no atomics, Context::flagStores), the plan kernel
    without reduce-and-forward fusion (one landing slot per channel), the
    plan kernel with nontemporal loads and write-through stores, and every
    engine with the system-scope flag sync instead of the default narrow one
    (DESIGN.md 4)."""
    k, v = knob.split("=")
    P = 3
    with tempfile.TemporaryDirectory() as d:
        env = rank_env(P)
        env[k] = v
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P), mode],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(P)]
        outs = []
        for p in procs:
            try:
                o, _ = p.communicate(timeout=240)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs.append(o.decode(errors="replace"))
        # every rank's output: the first rank to fail is often not rank 0
        every = "\n".join("---- rank %d (rc %s) ----\n%s" % (r, p.returncode, outs[r])
                          for r, p in enumerate(procs))
        for r, p in enumerate(procs):
            assert p.returncode == 0 and "OK" in outs[r], "rank %d failed:\n%s" % (r, every)


@pytest.mark.parametrize("P", [2, 3])
def test_link_probe_multiprocess(P):
    """The measured-link probe bench.py runs on the node (glx_link_probe):
    every rank's receive block through the context's canary-checked IPC path,
    ring and mesh patterns, DMA and copy-kernel writes, the busiest link's
    byte count; each peer's connect-time view (glx_context_peer_info); and an
    allreduce on the same context afterwards (the probe's blocks went back to
    the pool)."""
    with tempfile.TemporaryDirectory() as d:
        env = rank_env(P)
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P), "linkprobe"],
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
        every = "\n".join("---- rank %d (rc %s) ----\n%s" % (r, p.returncode, outs[r])
                          for r, p in enumerate(procs))
        for r, p in enumerate(procs):
            assert p.returncode == 0 and "OK" in outs[r], "rank %d failed:\n%s" % (r, every)


@pytest.mark.parametrize("P", [2, 4])
def test_algorithm_churn_multiprocess(P):
    """36 algorithms created, run twice and destroyed back to back per rank
    on every engine (one-shot, two-shot, plan kernel, host steps; ring and
    halving-doubling): shared blocks are pooled and reused across them while
    peers may still be finishing, so this checks the drain-before-reuse and
    pooling rules: bit-exact results, no fd growth."""
    with tempfile.TemporaryDirectory() as d:
        env = rank_env(P)
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P), "churn"],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(P)]
        outs = []
        for p in procs:
            try:
                o, _ = p.communicate(timeout=420 if P > 4 else 240)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs.append(o.decode(errors="replace"))
        for r, p in enumerate(procs):
            print(outs[r])
            assert p.returncode == 0, "rank %d failed:\n%s" % (r, outs[r])
            assert "OK" in outs[r]


def test_device_engine_timeout_raises_io_exception():
    """A device-driven kernel whose peers never arrive gives up after the
    context timeout (every wave exits), and run() raises IoException -- the
    one- and two-shot kernels and the DMA steps engine's flag waits."""
    P = 2
    with tempfile.TemporaryDirectory() as d:
        env = rank_env(P)
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P), "devtimeout"],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(P)]
        outs = []
        for p in procs:
            try:
                o, _ = p.communicate(timeout=120)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs.append(o.decode(errors="replace"))
        for r, p in enumerate(procs):
            print(outs[r])
            assert p.returncode == 0, "rank %d failed:\n%s" % (r, outs[r])
            assert "OK" in outs[r]


def test_dma_steps_copy_after_a_failed_credit_wait_is_reported_by_the_receiver():
    """a DMA steps copy enqueued behind a credit wait that
    gave up still runs; the receiver's run must fail (the sender's abort
    mark, kernels.h) instead of returning the overwritten region
    (mp_worker.py dmaabort)."""
    P = 2
    with tempfile.TemporaryDirectory() as d:
        env = rank_env(P)
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P), "dmaabort"],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(P)]
        outs = []
        for p in procs:
            try:
                o, _ = p.communicate(timeout=120)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs.append(o.decode(errors="replace"))
        for r, p in enumerate(procs):
            print(outs[r])
            assert p.returncode == 0, "rank %d failed:\n%s" % (r, outs[r])
            assert "OK" in outs[r]


@pytest.mark.parametrize("split", [2, 4])
@pytest.mark.parametrize("algo", [O.RING_CHUNKED, O.HALVING_DOUBLING, MESH],
                         ids=["ring_chunked", "halving_doubling", "mesh"])
def test_split_peer_copies(algo, split):
    """Each SEND split over several copy streams (parts >= 1 MiB) must give the
    same bits; the split is read when the algorithm is created."""
    import gloo_amd
    P, N = 3, (6 << 20) // 4 + 77
    ins = case_inputs(P, N, O.FLOAT32, 1, 0, seed=5)
    gloo_amd.set_copy_engine("dma", 64)
    gloo_amd.set_copy_split(split)
    try:
        out = gpu_allreduce(algo, O.SUM, O.FLOAT32, ins, runs=2)
    finally:
        gloo_amd.set_copy_split(1)
        gloo_amd.set_copy_engine("dma", 64)
    ref_algo = O.HALVING_DOUBLING if algo == O.HALVING_DOUBLING else O.RING_CHUNKED
    check_all(out, O.allreduce(ref_algo, O.SUM, O.FLOAT32, ins), O.FLOAT32, O.SUM)


@pytest.mark.parametrize("split", [1, 2])
@pytest.mark.parametrize("algo", [O.RING_CHUNKED, O.HALVING_DOUBLING, MESH],
                         ids=["ring_chunked", "halving_doubling", "mesh"])
def test_kernel_copy_engine(algo, split):
    """Peer copies made by the xGMI copy kernel instead of the DMA engines:
    same bits, including unaligned chunk boundaries (odd N)."""
    import gloo_amd
    P, N = 4, (3 << 20) // 4 + 13
    ins = case_inputs(P, N, O.FLOAT32, 1, 0, seed=9)
    gloo_amd.set_copy_engine("kernel", blocks=16)
    gloo_amd.set_copy_split(split)
    try:
        out = gpu_allreduce(algo, O.SUM, O.FLOAT32, ins, runs=2)
        out16 = gpu_allreduce(algo, O.SUM, O.FLOAT16,
                              case_inputs(3, 1001, O.FLOAT16, 1, 0, seed=2))
    finally:
        gloo_amd.set_copy_engine("dma", blocks=64)
        gloo_amd.set_copy_split(1)
    ref_algo = O.HALVING_DOUBLING if algo == O.HALVING_DOUBLING else O.RING_CHUNKED
    check_all(out, O.allreduce(ref_algo, O.SUM, O.FLOAT32, ins), O.FLOAT32, O.SUM)
    ins16 = case_inputs(3, 1001, O.FLOAT16, 1, 0, seed=2)
    check_all(out16, O.allreduce(ref_algo, O.SUM, O.FLOAT16, ins16), O.FLOAT16, O.SUM)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs in one process")
@pytest.mark.parametrize("algo", [O.RING_CHUNKED, O.HALVING_DOUBLING],
                         ids=["ring_chunked", "halving_doubling"])
def test_multi_device_pointers_in_one_rank(algo):
    """one rank's pointers on different GPUs (the reference's
    multi-device CUDA ranks): folded and broadcast over peer access."""
    import gloo_amd
    P, N, nptrs = 2, 100003, 2
    ins = case_inputs(P, N, O.FLOAT32, nptrs, 0, seed=14)
    store = gloo_amd.rendezvous.HashStore()
    bufs = [[torch.from_numpy(ins[r][i].copy()).to("cuda:%d" % i) for i in range(nptrs)]
            for r in range(P)]
    for d in range(nptrs):
        torch.cuda.synchronize(d)

    def rank_fn(r):
        ctx = gloo_amd.rendezvous.Context(r, P, 0)
        ctx.connectFullMesh(store)
        cls = (gloo_amd.AllreduceHalvingDoubling if algo == O.HALVING_DOUBLING
               else gloo_amd.AllreduceRingChunked)
        alg = cls(ctx, bufs[r])
        alg.run()
        alg.close()
        return True

    run_ranks(P, rank_fn)
    exp = O.allreduce(algo, O.SUM, O.FLOAT32, ins)
    for r in range(P):
        for i in range(nptrs):
            assert_same(bufs[r][i].cpu().numpy(), exp[r][i], O.FLOAT32, O.SUM)


@pytest.mark.parametrize("P", [2, 3, 4, 8])
@pytest.mark.parametrize("N", [1, 255, 1000, 4099, 100003])
def test_replicated_schedule_matches_ring_chunked_oracle(P, N):
    import gloo_amd  # noqa: F401
    ins = case_inputs(P, N, O.FLOAT32, 1, 0, seed=18)
    out = gpu_allreduce(REPL, O.SUM, O.FLOAT32, ins, runs=2)
    check_all(out, O.allreduce(O.RING_CHUNKED, O.SUM, O.FLOAT32, ins), O.FLOAT32, O.SUM)


@pytest.mark.parametrize("dtype,op", [(O.FLOAT16, O.SUM), (O.FLOAT32, O.MAX),
                                      (O.INT64, O.PRODUCT), (O.BFLOAT16, O.MIN)],
                         ids=lambda x: str(x))
def test_replicated_schedule_dtypes_multi_pointer(dtype, op):
    P, N = 5, 20011
    ins = case_inputs(P, N, dtype, 2, 0, seed=19)
    out = gpu_allreduce(REPL, op, dtype, ins, streams=True)
    check_all(out, O.allreduce(O.RING_CHUNKED, op, dtype, ins), dtype, op)


@pytest.mark.parametrize("P,N", [(2, 1000), (3, 70000), (4, 100003), (8, 4099)])
def test_auto_schedule_is_ring_chunked(P, N):
    """The default AllreduceRingChunked picks its data movement by size; the
    bits are the reference's whatever it picks."""
    ins = case_inputs(P, N, O.FLOAT32, 1, 0, seed=23)
    out = gpu_allreduce(AUTO, O.SUM, O.FLOAT32, ins, runs=2)
    check_all(out, O.allreduce(O.RING_CHUNKED, O.SUM, O.FLOAT32, ins), O.FLOAT32, O.SUM)


@pytest.mark.parametrize("algo", [O.RING_CHUNKED, O.HALVING_DOUBLING],
                         ids=["ring_chunked", "halving_doubling"])
def test_events_order_a_consumer_stream(algo):
    """gloo::CudaStream's record/wait (gloo/cuda.h:40-120) through the C ABI:
    the algorithm runs on a user stream; alg.record(ev) marks the end of its
    work; a second stream waits for the event on the device and copies the
    result out, with no host synchronisation in between."""
    import gloo_amd
    P, N = 3, 1 << 20
    ins = case_inputs(P, N, O.FLOAT32, 1, 0, seed=23)
    exp = O.allreduce(algo, O.SUM, O.FLOAT32, ins)
    store = gloo_amd.rendezvous.HashStore()
    bufs = [to_dev(ins[r][0], O.FLOAT32) for r in range(P)]
    outs = [torch.zeros(N, device="cuda") for _ in range(P)]
    torch.cuda.synchronize()
    cls = gloo_amd.AllreduceRingChunked if algo == O.RING_CHUNKED \
        else gloo_amd.AllreduceHalvingDoubling

    def rank_fn(r):
        ctx = gloo_amd.rendezvous.Context(r, P, 0)
        ctx.setTimeout(60)
        ctx.connectFullMesh(store)
        work, consumer = torch.cuda.Stream(), torch.cuda.Stream()
        kw = {"schedule": "ring"} if algo == O.RING_CHUNKED else {}
        alg = cls(ctx, [bufs[r]], streams=[work], **kw)
        ev = gloo_amd.Event()
        alg.run()
        alg.record(ev)
        ev.wait(consumer)                 # device-side wait, host not blocked
        with torch.cuda.stream(consumer):
            outs[r].copy_(bufs[r])
        ev2 = gloo_amd.Event()
        ev2.record(consumer)
        ev2.wait()                        # host waits for the consumer's copy
        assert ev.query() and ev2.query()
        alg.close()
        return True

    run_ranks(P, rank_fn, timeout=90)
    for r in range(P):
        assert_same(from_dev(outs[r], O.FLOAT32), exp[r][0], O.FLOAT32, O.SUM)


def test_transport_stats_name_the_mechanism():
    """transport_stats() says how messages moved: thread-ranks sharing one
    device copy with hipMemcpyAsync (device_copies), the copy kernel counts
    as kernel_copies, and the bytes match bytes_sent() per run."""
    import gloo_amd
    P, N = 2, 1 << 18
    ins = case_inputs(P, N, O.FLOAT32, 1, 0, seed=24)
    store = gloo_amd.rendezvous.HashStore()
    bufs = [to_dev(ins[r][0], O.FLOAT32) for r in range(P)]
    torch.cuda.synchronize()
    stats = {}

    def rank_fn(r, engine):
        ctx = gloo_amd.rendezvous.Context(r, P, 0)
        ctx.setTimeout(60)
        ctx.connectFullMesh(store)
        alg = gloo_amd.AllreduceRingChunked(ctx, [bufs[r]], schedule="ring")
        for _ in range(3):
            alg.run()
        stats[(r, engine)] = (alg.transport_stats(), alg.bytes_sent(), alg.engine())
        alg.close()
        return True

    # the copy engine is read at construction (process-wide setting)
    for engine in ("dma", "kernel"):
        store = gloo_amd.rendezvous.HashStore()
        gloo_amd.set_copy_engine(engine, 64)
        try:
            run_ranks(P, lambda r: rank_fn(r, engine), timeout=90)
        finally:
            gloo_amd.set_copy_engine("dma", 64)
    for r in range(P):
        st, sent, eng = stats[(r, "dma")]
        assert eng == "steps"
        assert st["peer_copies"] == 0 and st["device_copies"] > 0 and st["kernel_copies"] == 0
        assert st["bytes"] == 3 * sent
        st, sent, eng = stats[(r, "kernel")]
        assert st["kernel_copies"] > 0 and st["device_copies"] == 0
        assert st["bytes"] == 3 * sent


def test_dma_engine_falls_back_for_threads_sharing_a_device():
    """Rank threads of one process on one device share its hardware queues,
    where one rank's flag wait could hold up the very copy of a peer it waits
    for: asking for the DMA steps engine gives them host-issued steps
    (HipPlanExecutor::dmaStepsAvailable), with the same bits."""
    import gloo_amd
    P, N = 2, 100003
    ins = case_inputs(P, N, O.FLOAT32, 1, 0, seed=25)
    exp = O.allreduce(O.RING_CHUNKED, O.SUM, O.FLOAT32, ins)
    store = gloo_amd.rendezvous.HashStore()
    bufs = [to_dev(ins[r][0], O.FLOAT32) for r in range(P)]
    torch.cuda.synchronize()
    engines = {}

    def rank_fn(r):
        ctx = gloo_amd.rendezvous.Context(r, P, 0)
        ctx.setTimeout(60)
        ctx.connectFullMesh(store)
        alg = gloo_amd.AllreduceRingChunked(ctx, [bufs[r]], schedule="ring")
        engines[r] = alg.engine()
        alg.run()
        alg.close()
        return True

    gloo_amd.set_steps_engine("dma")
    try:
        run_ranks(P, rank_fn, timeout=90)
    finally:
        gloo_amd.set_steps_engine("auto")
    for r in range(P):
        assert engines[r] == "steps"
        assert np.array_equal(from_dev(bufs[r], O.FLOAT32).view(np.uint32),
                              exp[r][0].view(np.uint32))


def test_multidev_check_script_on_one_device():
    """tools/multidev_check.py -- what bench.py's N = 1 line runs on a box
    with several GPUs -- in its self-test mode: the same
    cases with every "device" being device 0, so the script's plumbing and
    checks are exercised on the one-GPU boxes too."""
    import json
    import subprocess
    import sys
    script = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                          "tools", "multidev_check.py")
    p = subprocess.run([sys.executable, script, "--same-device"], capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["ok"] is True and len(d["cases"]) == 6, d


@pytest.mark.parametrize("P,queues,mode,engine", [
    (8, "4", "shared", "steps"), (8, "1", "shared", "devsteps"), (4, "4", "shared", "devsteps"),
    (8, "1", None, "steps"), (4, "2", None, "steps")])
def test_device_engines_respect_the_shared_gpu_queue_budget(P, queues, mode, engine):
    """Processes sharing one GPU get the device engines only when they opt in
    (GLOO_AMD_DEVICE_ENGINES=shared) and only while ranks x
    (GPU_MAX_HW_QUEUES + 1) <= 20 (beyond the GPU's 24 user
    queues the scheduler time-slices them and every dependent step waits for
    a rotation).  Shared mode: 8 x 4 falls back to host-issued steps, 8 x 1
    and 4 x 4 keep the plan kernel.  The automatic mode (None) keeps ranks
    sharing a GPU on host-issued steps whatever the queue count (8 x 1 is
    the configuration that starved a GEMM, profiles/r9j_*, r9l_*).  Every
    rank agrees and the result is exact."""
    with tempfile.TemporaryDirectory() as d:
        env = dict(rank_env(P, device_engines=mode), GPU_MAX_HW_QUEUES=queues)
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P), "engine_choice"],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(P)]
        outs = []
        for p in procs:
            try:
                o, _ = p.communicate(timeout=240)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs.append(o.decode(errors="replace"))
        every = "\n".join("---- rank %d (rc %s) ----\n%s" % (r, p.returncode, outs[r])
                          for r, p in enumerate(procs))
        for r, p in enumerate(procs):
            assert p.returncode == 0 and "OK" in outs[r], "rank %d failed:\n%s" % (r, every)
            assert "ENGINE rank %d %s" % (r, engine) in outs[r], every
