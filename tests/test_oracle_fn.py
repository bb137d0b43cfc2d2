"""The oracle's restatement of gloo::allreduce(AllreduceOptions)
(oracle/gloo_oracle.c: oracle_allreduce_fn, following gloo/allreduce.cc)
pinned to the reference: the committed fixtures in
tests/golden/allreduce_fn_golden.* were produced by the reference's own
gloo::allreduce (tests/golden/make_golden.py), and, where the compiled
reference is present (this container), random cases are compared live."""
import numpy as np
import pytest

from helpers import (check_against_golden, fn_case_buffers, load_allreduce_fn_golden,
                     same_bits, sha)
from oracle import oracle as O

INDEX, DATA = load_allreduce_fn_golden()


@pytest.mark.parametrize("rec", INDEX, ids=[r["name"] for r in INDEX])
def test_oracle_fn_matches_reference_golden(rec):
    ins, outs = fn_case_buffers(rec)
    assert sha([x for row in ins + outs for x in row]) == rec["input_sha256"]
    res = O.allreduce_fn(rec["algo"], rec["op"], rec["dtype"], ins, outs,
                         rec["max_segment_size"])
    for r in range(rec["P"]):
        for i in range(rec["nout"]):
            assert same_bits(res[r][i], res[0][0]), (r, i)
    check_against_golden(rec, DATA, res[0][0])


@pytest.mark.parametrize("rec", [r for r in INDEX if r["dtype"] == O.UINT64 and r["N"] > 0],
                         ids=lambda r: r["name"])
def test_reference_test_closed_form(rec):
    """allreduce_test.cc:343-352: out[j][k] == k*stride^2 + stride(stride-1)/2."""
    P, N = rec["P"], rec["N"]
    nptrs = rec["nout"]
    stride = P * nptrs
    k = np.arange(N, dtype=np.uint64)
    exp = k * np.uint64(stride * stride) + np.uint64(stride * (stride - 1) // 2)
    if rec["name"] in DATA:
        assert np.array_equal(DATA[rec["name"]], exp)


@pytest.mark.skipif(not O.ref_available(), reason="compiled reference not present")
@pytest.mark.parametrize("algo", [O.FN_RING, O.FN_BCUBE])
@pytest.mark.parametrize("seed", range(6))
def test_oracle_fn_vs_live_reference(algo, seed):
    rng = np.random.default_rng(seed)
    P = int(rng.integers(2, 9))
    N = int(rng.integers(1, 3000))
    nin = int(rng.integers(0, 4))
    nout = int(rng.integers(1, 3))
    dtype = [O.FLOAT32, O.FLOAT16, O.INT32, O.FLOAT64][seed % 4]
    op = [O.SUM, O.MAX, O.MIN, O.PRODUCT][(seed // 2) % 4]
    ms = [0, 128, 1000][seed % 3]
    ins = [[O.fill(dtype, N, 0, seed=seed, rank=r, ptr_index=i) for i in range(nin)]
           for r in range(P)]
    outs = [[O.fill(dtype, N, 0, seed=seed + 99, rank=r, ptr_index=i) for i in range(nout)]
            for r in range(P)]
    a = O.allreduce_fn(algo, op, dtype, ins, outs, ms)
    b = O.allreduce_fn(algo, op, dtype, ins, outs, ms, use_ref=True)
    for r in range(P):
        for i in range(nout):
            assert same_bits(a[r][i], b[r][i]), (r, i)
