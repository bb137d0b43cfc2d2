"""GPU tests of the round-4 widening OUTSIDE the SURVEY 8 contract:
gloo::AllreduceRing<T>, gloo::AllreduceBcube<T> (the class) and
gloo::AllreduceLocal<T> -- SURVEY 2.1 lists these schedules as out of scope
("Other allreduce schedules ... not named in north_star").  The code stays;
its tests carry the `widening` marker instead of `gpu`, so `pytest -m gpu`
(the hot path's suite) does not spend GPU time on them.  Run them with
`pytest -m widening` on a GPU box; they are skipped without a GPU."""
import numpy as np
import pytest

from helpers import case_inputs, check_ring_against_golden, load_ring_golden, run_ranks
from oracle import oracle as O

pytestmark = pytest.mark.widening

torch = pytest.importorskip("torch")

from test_allreduce_gpu import check_all, gpu_allreduce  # noqa: E402
from test_reduce_gpu import assert_same, from_dev, to_dev  # noqa: E402


# gloo::AllreduceRing<T> (gloo/allreduce_ring.h): every rank's own result
# against the compiled reference's per-rank outputs (float results differ
# between ranks, tests/golden/allreduce_ring_golden.json), the reference
# test's grid (allreduce_test.cc:241-249, P = 1..15), dtypes x ops, several
# pointers with streams.
RING_INDEX, RING_DATA = load_ring_golden()


@pytest.mark.parametrize("rec", RING_INDEX, ids=[r["name"] for r in RING_INDEX])
def test_allreduce_ring_vs_reference_golden(rec):
    ins = case_inputs(rec["P"], rec["N"], rec["dtype"], rec["nptrs"], rec["kind"], rec["seed"])
    out = gpu_allreduce(O.RING, rec["op"], rec["dtype"], ins, runs=2)
    check_ring_against_golden(rec, RING_DATA, out)


@pytest.mark.parametrize("P", list(range(1, 16)))
@pytest.mark.parametrize("N", [0, 4, 100, 1000, 10000])
def test_allreduce_ring_reference_test_grid(P, N):
    ins = [[np.full(N, r, dtype=np.float32)] for r in range(P)]
    out = gpu_allreduce(O.RING, O.SUM, O.FLOAT32, ins, runs=2)
    for r in range(P):
        assert np.all(out[r][0] == P * (P - 1) // 2), "rank %d" % r


@pytest.mark.parametrize("dtype", [O.INT8, O.INT32, O.INT64, O.UINT64, O.FLOAT64, O.FLOAT16,
                                   O.BFLOAT16], ids=lambda d: O.DTYPE_NAMES[d])
@pytest.mark.parametrize("op", [O.SUM, O.PRODUCT, O.MAX, O.MIN],
                         ids=lambda o: O.OP_NAMES[o])
def test_allreduce_ring_dtypes_ops(dtype, op):
    ins = case_inputs(4, 4099, dtype, 1, 0, seed=33)
    out = gpu_allreduce(O.RING, op, dtype, ins)
    check_all(out, O.allreduce(O.RING, op, dtype, ins), dtype, op)


@pytest.mark.parametrize("P,nptrs", [(1, 3), (3, 2), (5, 2)])
def test_allreduce_ring_multi_pointer_streams(P, nptrs):
    ins = case_inputs(P, 100003, O.FLOAT32, nptrs, 0, seed=34)
    out = gpu_allreduce(O.RING, O.SUM, O.FLOAT32, ins, runs=2, streams=True)
    check_all(out, O.allreduce(O.RING, O.SUM, O.FLOAT32, ins), O.FLOAT32, O.SUM)


# gloo::AllreduceBcube<T> (gloo/allreduce_bcube.h): groups of the context's
# base ranks; the reference's per-rank outputs, its test grid (allreduce_
# test.cc:271-299), dtypes x ops.
BCUBE_INDEX, BCUBE_DATA = load_ring_golden("bcube")


@pytest.mark.parametrize("rec", BCUBE_INDEX, ids=[r["name"] for r in BCUBE_INDEX])
def test_allreduce_bcube_vs_reference_golden(rec):
    ins = case_inputs(rec["P"], rec["N"], rec["dtype"], rec["nptrs"], rec["kind"], rec["seed"])
    out = gpu_allreduce(O.BCUBE, rec["op"], rec["dtype"], ins, runs=2, base=rec["base"])
    check_ring_against_golden(rec, BCUBE_DATA, out)


BCUBE_REF_GRID = ([(2, P) for P in (1, 2, 4, 8, 16)] + [(3, P) for P in (1, 3, 9, 27)] +
                  [(4, P) for P in (1, 4, 16)])


@pytest.mark.parametrize("base,P", BCUBE_REF_GRID, ids=["b%d-P%d" % g for g in BCUBE_REF_GRID])
@pytest.mark.parametrize("N", [0, 1, 64, 1000])
def test_allreduce_bcube_reference_test_grid(base, P, N):
    ins = [[np.full(N, r, dtype=np.float32)] for r in range(P)]
    out = gpu_allreduce(O.BCUBE, O.SUM, O.FLOAT32, ins, runs=2, base=base)
    for r in range(P):
        assert np.all(out[r][0] == P * (P - 1) // 2), "rank %d" % r


@pytest.mark.parametrize("dtype", [O.INT8, O.INT64, O.FLOAT64, O.FLOAT16, O.BFLOAT16],
                         ids=lambda d: O.DTYPE_NAMES[d])
@pytest.mark.parametrize("op", [O.SUM, O.PRODUCT, O.MAX, O.MIN],
                         ids=lambda o: O.OP_NAMES[o])
def test_allreduce_bcube_dtypes_ops(dtype, op):
    ins = case_inputs(6, 4099, dtype, 1, 0, seed=35)
    out = gpu_allreduce(O.BCUBE, op, dtype, ins, base=3)
    check_all(out, O.allreduce(O.BCUBE, op, dtype, ins, base=3), dtype, op)


@pytest.mark.parametrize("P,nptrs", [(1, 1), (1, 3), (3, 2), (4, 4)])
@pytest.mark.parametrize("dtype,op", [(O.FLOAT32, O.SUM), (O.FLOAT16, O.SUM), (O.INT32, O.MAX)],
                         ids=str)
def test_allreduce_local(P, nptrs, dtype, op):
    """gloo::AllreduceLocal<T> (gloo/allreduce_local.cc:21-31): each rank's
    own pointers folded and broadcast; ranks do not exchange anything."""
    import gloo_amd
    ins = case_inputs(P, 100003, dtype, nptrs, 0, seed=36)
    store = gloo_amd.rendezvous.HashStore()
    bufs = [[to_dev(x, dtype) for x in row] for row in ins]
    torch.cuda.synchronize()

    def rank_fn(r):
        ctx = gloo_amd.rendezvous.Context(r, P, 0)
        ctx.connectFullMesh(store)
        alg = gloo_amd.AllreduceLocal(ctx, [b.data_ptr() for b in bufs[r]], 100003,
                                      gloo_amd.ReductionFunction(op), dtype=dtype)
        alg.run()
        alg.close()
        return True

    run_ranks(P, rank_fn, timeout=90)
    torch.cuda.synchronize()
    for r in range(P):
        exp = O.allreduce(O.RING_CHUNKED, op, dtype, [ins[r]])[0]  # one rank's fold
        for i in range(nptrs):
            assert_same(from_dev(bufs[r][i], dtype), exp[i], dtype, op)
