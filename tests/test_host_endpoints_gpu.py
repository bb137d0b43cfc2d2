"""Host-memory endpoints: the class algorithms on buffers in
host memory -- the reference's own calling convention, AllreduceRingChunked<T>
(ctx, {host ptr}, count) -- staged through the GPU: H2D in first-use order,
the schedule on device copies, each range copied back after its final write.
Results must be the reference's bits (oracle), for pageable numpy buffers and
pinned torch buffers."""
import numpy as np
import pytest

from helpers import case_inputs, run_ranks, same_bits
from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ALGOS = {"ring_chunked": O.RING_CHUNKED, "halving_doubling": O.HALVING_DOUBLING,
         "ring_chunked_mesh": O.RING_CHUNKED}


def make(gloo_amd, algo, ctx, bufs, op, dtype=None):
    fn = {O.SUM: gloo_amd.ReductionFunction.sum, O.MAX: gloo_amd.ReductionFunction.max,
          O.MIN: gloo_amd.ReductionFunction.min,
          O.PRODUCT: gloo_amd.ReductionFunction.product}[op]
    if algo == "halving_doubling":
        return gloo_amd.AllreduceHalvingDoubling(ctx, bufs, fn=fn, dtype=dtype)
    return gloo_amd.AllreduceRingChunked(
        ctx, bufs, fn=fn, schedule="mesh" if algo == "ring_chunked_mesh" else "ring",
        dtype=dtype)


def host_allreduce(algo, op, dtype, inputs, runs=1, pinned=False, stats=None):
    import gloo_amd
    P = len(inputs)
    store = gloo_amd.rendezvous.HashStore()
    if pinned:
        tv = {O.FLOAT32: torch.float32, O.INT32: torch.int32, O.FLOAT16: torch.float16,
              O.FLOAT64: torch.float64}[dtype]
        bufs = [[torch.from_numpy(x.copy()).view(tv).pin_memory() for x in row]
                for row in inputs]
    else:
        bufs = [[np.array(x, copy=True) for x in row] for row in inputs]

    def rank_fn(r):
        ctx = gloo_amd.rendezvous.Context(r, P, 0)
        ctx.setTimeout(60)
        ctx.connectFullMesh(store)
        alg = make(gloo_amd, algo, ctx, bufs[r], op,
                   dtype if dtype in (O.FLOAT16, O.BFLOAT16) and not pinned else None)
        for k in range(runs):
            if k > 0:  # the host buffers are the algorithm's: refill in place
                for b, x in zip(bufs[r], inputs[r]):
                    if pinned:
                        b.copy_(torch.from_numpy(x.copy()).view(b.dtype))
                    else:
                        b[...] = x
            alg.run()
        if stats is not None:
            stats[r] = alg.transport_stats()
        alg.close()
        return True

    run_ranks(P, rank_fn, timeout=120)
    if pinned:
        return [[b.view(torch.uint8).numpy().view(O.NP_DTYPE[dtype]).copy() for b in row]
                for row in bufs]
    return bufs


def check(out, exp):
    for r in range(len(exp)):
        for i in range(len(exp[r])):
            assert same_bits(out[r][i], exp[r][i]), (r, i)


@pytest.mark.parametrize("algo", list(ALGOS))
@pytest.mark.parametrize("P,N", [(1, 1000), (2, 1), (2, 100003), (3, 4099), (4, 1 << 20),
                                 (5, 3 << 20), (8, (2 << 20) + 5)])
def test_pageable_host_buffers_vs_oracle(algo, P, N):
    ins = case_inputs(P, N, O.FLOAT32, 1, 0, seed=3)
    out = host_allreduce(algo, O.SUM, O.FLOAT32, ins, runs=2)
    check(out, O.allreduce(ALGOS[algo], O.SUM, O.FLOAT32, ins))


@pytest.mark.parametrize("algo", list(ALGOS))
@pytest.mark.parametrize("dtype,op", [(O.FLOAT16, O.SUM), (O.INT32, O.MAX),
                                      (O.FLOAT64, O.PRODUCT)], ids=str)
def test_pinned_multi_pointer_host_buffers(algo, dtype, op):
    P, N = 3, 300007
    ins = case_inputs(P, N, dtype, 2, 0, seed=4)
    out = host_allreduce(algo, op, dtype, ins, runs=2, pinned=True)
    check(out, O.allreduce(ALGOS[algo], op, dtype, ins))


@pytest.mark.parametrize("pinned", [True, False], ids=["pinned", "pageable"])
@pytest.mark.parametrize("dtype,op,nptrs", [(O.FLOAT32, O.SUM, 2), (O.FLOAT16, O.SUM, 3),
                                            (O.INT32, O.MAX, 2)], ids=str)
def test_single_rank_multi_pointer_host_pipelined(pinned, dtype, op, nptrs):
    """One rank, several host pointers above kOnDeviceThreshold: the fold
    runs per 8 MiB staging piece (H2D, fold, D2H to every pointer,
    overlapped); several pieces and a ragged last one, two runs."""
    N = (5 << 20) + 4099
    ins = case_inputs(1, N, dtype, nptrs, 0, seed=61)
    out = host_allreduce("ring_chunked", op, dtype, ins, runs=2, pinned=pinned)
    check(out, O.allreduce(O.RING_CHUNKED, op, dtype, ins))


def test_freed_uncached_blocks_do_not_poison_later_allocations():
    """memory freed with hipFree after an uncached allocation
    came back broken from later plain hipMalloc calls (wrong results in
    later host-memory runs of the same process).  Contexts here create and
    destroy uncached receive regions, and every later run -- including a
    one-rank run whose staging buffers are plain hipMalloc memory -- must
    still be exact; the executor keeps freed uncached blocks in a
    process-wide cache instead of handing them back.  Alone this test does
    not reproduce the hazard; this FILE does: with GLOO_AMD_UC_CACHE=0 (the
    blocks hipFree'd) 10 of its cases fail, this one included, and with the
    cache none (profiles/r3j_*)."""
    sizes = (100003, 300007, 1 << 20, 65539, (1 << 21) + 5, 300007, 4099, 1 << 19)
    for rep, n in enumerate(sizes):
        algo = ("ring_chunked", "halving_doubling", "ring_chunked_mesh")[rep % 3]
        ins = case_inputs(3, n, O.FLOAT64, 2, 0, seed=70 + rep)
        out = host_allreduce(algo, O.PRODUCT, O.FLOAT64, ins, runs=2, pinned=True)
        check(out, O.allreduce(ALGOS[algo], O.PRODUCT, O.FLOAT64, ins))
        ins1 = case_inputs(1, (5 << 20) + 4099, O.FLOAT32, 2, 0, seed=80 + rep)
        out1 = host_allreduce("ring_chunked", O.SUM, O.FLOAT32, ins1, runs=2,
                              pinned=rep % 2 == 0)
        check(out1, O.allreduce(O.RING_CHUNKED, O.SUM, O.FLOAT32, ins1))


def test_single_rank_multi_pointer_host():
    ins = case_inputs(1, 5000, O.FLOAT32, 3, 0, seed=6)
    out = host_allreduce("ring_chunked", O.SUM, O.FLOAT32, ins)
    check(out, O.allreduce(O.RING_CHUNKED, O.SUM, O.FLOAT32, ins))


def test_mixed_host_and_device_buffers_are_rejected():
    import gloo_amd
    ctx = gloo_amd.rendezvous.Context(0, 1, 0)
    with pytest.raises(gloo_amd.EnforceNotMet):
        gloo_amd.AllreduceRingChunked(ctx, [np.zeros(64, np.float32),
                                            torch.zeros(64, device="cuda")])


@pytest.mark.parametrize("algo", ["ring_chunked", "halving_doubling"])
@pytest.mark.parametrize("dtype,op", [(O.FLOAT32, O.SUM), (O.FLOAT16, O.SUM),
                                      (O.FLOAT16, O.MAX), (O.INT8, O.PRODUCT),
                                      (O.BFLOAT16, O.SUM), (O.UINT64, O.MIN)], ids=str)
@pytest.mark.parametrize("nptrs", [2, 3])
def test_on_device_threshold(algo, dtype, op, nptrs):
    """kOnDeviceThreshold (gloo/algorithm.cc:16): host buffers of several
    pointers below 256 KiB are folded on the host and staged as one buffer
    (the reference's cudaHostReduce/cudaHostBroadcast,
    gloo/cuda_allreduce_halving_doubling.cc:478-484); at and above it the
    fold runs on the device.  Same bits either way."""
    es = {O.FLOAT32: 4, O.FLOAT16: 2, O.BFLOAT16: 2, O.INT8: 1, O.UINT64: 8}[dtype]
    P = 2
    for nbytes, host in ((64 << 10, True), ((256 << 10) - 16, True), (256 << 10, False),
                         ((256 << 10) + 4096, False)):
        N = nbytes // es
        ins = case_inputs(P, N, dtype, nptrs, 0, seed=9)
        stats = {}
        out = host_allreduce(algo, op, dtype, ins, runs=2, stats=stats)
        check(out, O.allreduce(ALGOS[algo], op, dtype, ins))
        for r in range(P):
            assert (stats[r]["host_folds"] == 2) == host, (nbytes, stats[r])


@pytest.fixture
def bounce_only():
    """Every pageable buffer of algorithms created meanwhile goes through the
    8 MiB bounce block instead of a pinned mirror of its size -- what the
    product does when the runtime cannot pin a whole mirror."""
    import gloo_amd
    gloo_amd.set_pinned_mirror_limit(4096)
    try:
        yield
    finally:
        gloo_amd.set_pinned_mirror_limit(0)


@pytest.mark.parametrize("algo", list(ALGOS))
@pytest.mark.parametrize("P,N", [(1, 1000), (2, 100003), (3, (5 << 20) + 3)])
def test_pageable_through_bounce_block(bounce_only, algo, P, N):
    ins = case_inputs(P, N, O.FLOAT32, 1, 0, seed=71)
    out = host_allreduce(algo, O.SUM, O.FLOAT32, ins, runs=2)
    check(out, O.allreduce(ALGOS[algo], O.SUM, O.FLOAT32, ins))


@pytest.mark.parametrize("dtype,op,nptrs", [(O.FLOAT32, O.SUM, 2), (O.FLOAT16, O.SUM, 3)],
                         ids=str)
def test_single_rank_multi_pointer_through_bounce_block(bounce_only, dtype, op, nptrs):
    N = (5 << 20) + 4099
    ins = case_inputs(1, N, dtype, nptrs, 0, seed=72)
    out = host_allreduce("ring_chunked", op, dtype, ins, runs=2)
    check(out, O.allreduce(O.RING_CHUNKED, op, dtype, ins))


@pytest.mark.parametrize("nin,nout", [(0, 1), (1, 1), (2, 2)])
def test_fn_host_buffers_through_bounce_block(bounce_only, nin, nout):
    """gloo_amd.allreduce on pageable host buffers: the staged path (one
    input or in place, one output) and the whole-buffer path (several)."""
    from test_allreduce_fn_gpu import host_allreduce_fn
    P, N = 3, (3 << 20) + 5
    data = case_inputs(P, N, O.FLOAT32, max(nin, nout), 0, seed=73)
    if nin == 0:
        ins, outs = [[] for _ in range(P)], [row[:nout] for row in data]
    else:
        ins = [row[:nin] for row in data]
        outs = [[np.zeros(N, np.float32) for _ in range(nout)] for _ in range(P)]
    got = host_allreduce_fn(1, O.SUM, O.FLOAT32, ins, outs, runs=2)
    exp = O.allreduce_fn(O.FN_RING, O.SUM, O.FLOAT32, ins, outs)
    for r in range(P):
        for i in range(nout):
            assert np.array_equal(got[r][i].view(np.uint32), exp[r][i].view(np.uint32)), (r, i)


def _hip_memory_type(ptr):
    """hipPointerGetAttributes(ptr).type through the HIP runtime the library
    uses: 1 = hipMemoryTypeHost (pinned or registered), anything else (or an
    error) = memory the runtime does not know."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    attr = (ctypes.c_byte * 128)()
    rc = hip.hipPointerGetAttributes(ctypes.byref(attr), ctypes.c_void_p(ptr))
    if rc != 0:
        hip.hipGetLastError()
        return None
    return ctypes.cast(attr, ctypes.POINTER(ctypes.c_int))[0]


@pytest.mark.parametrize("limit", [0, 4096], ids=["mirror", "bounce"])
def test_caller_pages_stay_unregistered(limit):
    """while an algorithm lives on a pageable host buffer, and
    after it ran, the caller's pages are unknown to the HIP runtime (no
    hipHostRegister of caller memory: the round-3 illegal address)."""
    import gloo_amd
    P, N = 2, (1 << 20) + 7
    ins = case_inputs(P, N, O.FLOAT32, 1, 0, seed=74)
    bufs = [np.array(row[0], copy=True) for row in ins]
    store = gloo_amd.rendezvous.HashStore()
    kinds = {}
    gloo_amd.set_pinned_mirror_limit(limit)
    try:
        def rank_fn(r):
            ctx = gloo_amd.rendezvous.Context(r, P, 0)
            ctx.setTimeout(60)
            ctx.connectFullMesh(store)
            alg = gloo_amd.AllreduceRingChunked(ctx, [bufs[r]], schedule="ring")
            alg.run()
            kinds[r] = (_hip_memory_type(bufs[r].ctypes.data),
                        _hip_memory_type(bufs[r].ctypes.data + 4 * (N - 1)))
            alg.close()
            ctx.close()
            return True
        run_ranks(P, rank_fn, timeout=120)
    finally:
        gloo_amd.set_pinned_mirror_limit(0)
    assert all(k != 1 for r in range(P) for k in kinds[r]), kinds
    check([[b] for b in bufs], O.allreduce(O.RING_CHUNKED, O.SUM, O.FLOAT32, ins))
