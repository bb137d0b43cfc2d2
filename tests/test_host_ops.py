"""CPU: the product's host-side local reduce (glx_host_reduce_n, the
cudaHostReduce analog used below kOnDeviceThreshold) against the reference's
own known answers (tests/golden/reduce_kats.npz: gloo/math.h run in place,
generated from oracle/_ref) and against the oracle for seeded k-way folds.
No GPU needed."""
import os

import numpy as np
import pytest

import gloo_amd
from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
KATS = np.load(os.path.join(HERE, "golden", "reduce_kats.npz"))
DTYPES = [O.INT8, O.UINT8, O.INT32, O.INT64, O.UINT64, O.FLOAT32, O.FLOAT64, O.FLOAT16]
OPS = [O.SUM, O.PRODUCT, O.MAX, O.MIN]


def same(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint8),
                          np.ascontiguousarray(b).view(np.uint8))


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("op", OPS)
def test_host_fold_matches_reference_kats(dtype, op):
    key = "reduce_%s_%s" % (O.DTYPE_NAMES[dtype], O.OP_NAMES[op])
    a, b = KATS[key + "_a"], KATS[key + "_b"]
    for x, y, want in ((a, b, KATS[key + "_ab"]), (b, a, KATS[key + "_ba"])):
        dst = np.array(x, copy=True)
        gloo_amd.math.host_reduce_n(op, dtype, dst, [dst, y])
        if dtype in (O.FLOAT32, O.FLOAT64) and op in (O.SUM, O.PRODUCT):
            # NaN payloads may differ (x86 propagation vs the fixture's); both NaN
            nan = np.isnan(want)
            assert np.array_equal(np.isnan(dst), nan)
            assert same(dst[~nan], want[~nan])
        else:
            assert same(dst, want), key


@pytest.mark.parametrize("dtype", DTYPES + [O.BFLOAT16])
@pytest.mark.parametrize("op", OPS)
@pytest.mark.parametrize("k", [2, 3, 5])
def test_host_fold_k_way_matches_oracle(dtype, op, k):
    n = 4099
    srcs = [O.fill(dtype, n, 0, seed=77, rank=j) for j in range(k)]
    exp = np.array(srcs[0], copy=True)
    for j in range(1, k):
        exp = O.reduce(op, dtype, exp, srcs[j])
    dst = np.zeros_like(srcs[0])
    gloo_amd.math.host_reduce_n(op, dtype, dst, srcs)
    assert same(dst, exp)


def test_f16_conversion_sweep_through_sum():
    """Every float16 sum rounds with cpu_float2half_rn: fold a + 0 (exact) and
    a + b over all 65536 x a few b and compare with the oracle's restatement
    (pinned to the reference by the golden conversion sweep)."""
    a = np.arange(65536, dtype=np.uint16)
    for bv in (0x0000, 0x3c00, 0x0001, 0x8001, 0x7bff, 0xfc00):
        b = np.full(65536, bv, dtype=np.uint16)
        dst = np.array(a, copy=True)
        gloo_amd.math.host_reduce_n(O.SUM, O.FLOAT16, dst, [dst, b])
        assert same(dst, O.reduce(O.SUM, O.FLOAT16, a, b))


def test_threshold_constant():
    # gloo/algorithm.cc:16 -- host reduce/bcast below 256 KiB
    from gloo_amd import _lib
    assert _lib.lib.glx_host_reduce_n is not None
