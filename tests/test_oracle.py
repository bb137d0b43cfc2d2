"""CPU: the oracle pinned against the reference (golden fixtures produced by
the reference itself, tests/golden/make_golden.py) and against the
reference test-suite's own known answers."""
import numpy as np
import pytest

from helpers import (GOLDEN, case_inputs, check_against_golden, check_ring_against_golden,
                     load_allreduce_golden, load_ring_golden, sha)
from oracle import oracle as O

INDEX, DATA = load_allreduce_golden()


@pytest.mark.parametrize("rec", INDEX, ids=[r["name"] for r in INDEX])
def test_oracle_allreduce_matches_reference_golden(rec):
    ins = case_inputs(rec["P"], rec["N"], rec["dtype"], rec["nptrs"], rec["kind"], rec["seed"])
    assert sha([x for row in ins for x in row]) == rec["input_sha256"], "input generator drift"
    out = O.allreduce(rec["algo"], rec["op"], rec["dtype"], ins)
    for r in range(rec["P"]):
        for i in range(rec["nptrs"]):
            check_against_golden(rec, DATA, out[r][i])


def _reduce_kats():
    d = np.load(GOLDEN + "/reduce_kats.npz")
    keys = sorted({k.rsplit("_", 1)[0] for k in d.files if k.endswith("_a")})
    return d, keys


KATS, KAT_KEYS = _reduce_kats()
DT = {v: k for k, v in O.DTYPE_NAMES.items()}
OPS = {v: k for k, v in O.OP_NAMES.items()}


@pytest.mark.parametrize("key", KAT_KEYS)
def test_oracle_reduce_matches_reference(key):
    _, dname, oname = key.split("_")
    dtype, op = DT[dname], OPS[oname]
    a, b = KATS[key + "_a"], KATS[key + "_b"]
    def same(x, y):
        return np.array_equal(x.view(np.uint8), y.view(np.uint8))
    assert same(O.reduce(op, dtype, a, b), KATS[key + "_ab"])
    assert same(O.reduce(op, dtype, b, a), KATS[key + "_ba"])
    assert same(O.reduce(op, dtype, a, b, inplace=False), KATS[key + "_ab0"])
    assert same(O.reduce(op, dtype, b, a, inplace=False), KATS[key + "_ba0"])


def test_oracle_f16_conversions_match_reference():
    d = np.load(GOLDEN + "/f16_conversions.npz")
    f = d["f32_bits"].view(np.float32)
    assert np.array_equal(O.f32_to_f16(f), d["f16"])
    back = O.f16_to_f32(d["half_bits"]).view(np.uint32)
    assert np.array_equal(back, d["half_to_f32_bits"])


# gloo/test/math_test.cc:55-143 -- Sum/Product/Min/Max KATs, both orders.
@pytest.mark.parametrize("dtype", [O.INT8, O.UINT8, O.INT32, O.INT64, O.UINT64,
                                   O.FLOAT32, O.FLOAT64, O.FLOAT16])
def test_math_kats(dtype):
    num = 64

    def val(x):
        if dtype == O.FLOAT16:
            return O.f32_to_f16(np.array([x], dtype=np.float32))[0]
        return x

    cases = [(O.SUM, 2, 1, 1, 3, 2), (O.PRODUCT, 4, 2, 2, 8, 4), (O.MIN, 1, 2, 3, 1, 2),
             (O.MAX, 4, 2, 3, 4, 3)]
    for op, special, a0, b0, exp_special, exp_other in cases:
        for i in (0, 17, num - 1):
            a = np.full(num, val(a0), dtype=O.NP_DTYPE[dtype])
            b = np.full(num, val(b0), dtype=O.NP_DTYPE[dtype])
            a[i] = val(special)
            for x, y in ((a, b), (b, a)):
                c = O.reduce(op, dtype, x, y, inplace=False)
                exp = np.full(num, val(exp_other), dtype=O.NP_DTYPE[dtype])
                exp[i] = val(exp_special)
                assert np.array_equal(c, exp)


# gloo/test/allreduce_test.cc:143-169,251-269 -- SinglePointer: value = rank,
# every element must equal P(P-1)/2 exactly.
@pytest.mark.parametrize("P", list(range(1, 16)))
@pytest.mark.parametrize("N", [0, 4, 100, 1000, 10000])
def test_single_pointer_ring_chunked(P, N):
    ins = [[np.full(N, r, dtype=np.float32)] for r in range(P)]
    out = O.allreduce(O.RING_CHUNKED, O.SUM, O.FLOAT32, ins)
    for r in range(P):
        assert np.all(out[r][0] == P * (P - 1) // 2)


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 6, 7, 8, 9, 13, 16, 24, 32])
@pytest.mark.parametrize("N", [0, 1, 64, 1000])
def test_single_pointer_halving_doubling(P, N):
    ins = [[np.full(N, r, dtype=np.float32)] for r in range(P)]
    out = O.allreduce(O.HALVING_DOUBLING, O.SUM, O.FLOAT32, ins)
    for r in range(P):
        assert np.all(out[r][0] == P * (P - 1) // 2)


# gloo/test/base_test.h:184-235,420-460 -- stride pattern, rel 1e-4 (float),
# 1e-3 (float16, gloo/test/base_test.h:307-350).
@pytest.mark.parametrize("algo", [O.RING_CHUNKED, O.HALVING_DOUBLING])
@pytest.mark.parametrize("P,nptrs", [(2, 1), (3, 2), (4, 3), (7, 1)])
def test_stride_pattern(algo, P, nptrs):
    N = 1000
    ins = case_inputs(P, N, O.FLOAT32, nptrs, 1)
    out = O.allreduce(algo, O.SUM, O.FLOAT32, ins)
    stride = P * nptrs
    exp = np.arange(N, dtype=np.float64) * stride * stride + stride * (stride - 1) / 2
    for r in range(P):
        for i in range(nptrs):
            np.testing.assert_allclose(out[r][i], exp, rtol=1e-4)


@pytest.mark.parametrize("algo", [O.RING_CHUNKED, O.HALVING_DOUBLING])
def test_half_precision_reference_kat(algo):
    # gloo/test/allreduce_test.cc:212-239: fp16, P=4, N=1024, value = rank
    P, N = 4, 1024
    ins = [[O.fill(O.FLOAT16, N, 2, val=r)] for r in range(P)]
    out = O.allreduce(algo, O.SUM, O.FLOAT16, ins)
    exp = O.f32_to_f16(np.array([P * (P - 1) / 2], dtype=np.float32))[0]
    for r in range(P):
        assert np.all(out[r][0] == exp)


def test_reduction_order_ring_chunked():
    # element i of chunk c (owner r0 = c // 2) is
    # ((x[r0] + x[r0+1]) + ...) + x[r0+P-1] evaluated left to right in fp32.
    P, N = 5, 4099
    ins = case_inputs(P, N, O.FLOAT32, 1, 0)
    out = O.allreduce(O.RING_CHUNKED, O.SUM, O.FLOAT32, ins)[0][0]
    chunk = max(256, -(-N // (2 * P)))
    exp = np.empty(N, dtype=np.float32)
    for i in range(N):
        r0 = (i // chunk) // 2
        acc = np.float32(ins[r0][0][i])
        for k in range(1, P):
            acc = np.float32(acc + ins[(r0 + k) % P][0][i])
        exp[i] = acc
    assert np.array_equal(out, exp)


def test_reduction_order_halving_doubling():
    # P=8 -> ((x0+x1)+(x2+x3))+((x4+x5)+(x6+x7)), bit-exact
    P, N = 8, 1000
    ins = case_inputs(P, N, O.FLOAT32, 1, 0)
    x = [ins[r][0] for r in range(P)]
    exp = ((x[0] + x[1]) + (x[2] + x[3])) + ((x[4] + x[5]) + (x[6] + x[7]))
    out = O.allreduce(O.HALVING_DOUBLING, O.SUM, O.FLOAT32, ins)[0][0]
    assert np.array_equal(out, exp.astype(np.float32))


RING_INDEX, RING_DATA = load_ring_golden()


@pytest.mark.parametrize("rec", RING_INDEX, ids=[r["name"] for r in RING_INDEX])
def test_oracle_allreduce_ring_matches_reference_golden(rec):
    """gloo::AllreduceRing<T> (gloo/allreduce_ring.h:72-114): the oracle's
    restatement against the compiled reference's per-rank outputs."""
    ins = case_inputs(rec["P"], rec["N"], rec["dtype"], rec["nptrs"], rec["kind"])
    assert sha([x for row in ins for x in row]) == rec["input_sha256"]
    out = O.allreduce(O.RING, rec["op"], rec["dtype"], ins)
    for r in range(rec["P"]):
        for i in range(1, rec["nptrs"]):
            assert np.array_equal(out[r][i].view(np.uint8), out[r][0].view(np.uint8))
    check_ring_against_golden(rec, RING_DATA, out)


def test_allreduce_ring_ranks_differ_for_floats():
    """The reference's AllreduceRing leaves each rank its own summation order:
    with seeded fp32 inputs at P = 8 the ranks' results are not all equal
    (which is why its fixtures hold every rank's digest)."""
    rec = next(r for r in RING_INDEX if r["P"] == 8 and r["N"] == 100003 and r["kind"] == 0)
    assert len(set(rec["output_sha256"])) > 1


BCUBE_INDEX, BCUBE_DATA = load_ring_golden("bcube")


@pytest.mark.parametrize("rec", BCUBE_INDEX, ids=[r["name"] for r in BCUBE_INDEX])
def test_oracle_allreduce_bcube_matches_reference_golden(rec):
    """gloo::AllreduceBcube<T> (gloo/allreduce_bcube.h:256-695) with the
    context's base: the oracle's restatement against the compiled
    reference's per-rank outputs."""
    ins = case_inputs(rec["P"], rec["N"], rec["dtype"], rec["nptrs"], rec["kind"])
    assert sha([x for row in ins for x in row]) == rec["input_sha256"]
    out = O.allreduce(O.BCUBE, rec["op"], rec["dtype"], ins, base=rec["base"])
    check_ring_against_golden(rec, BCUBE_DATA, out)
