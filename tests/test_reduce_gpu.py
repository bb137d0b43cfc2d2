"""GPU parity of the per-chunk reduction kernel (glx_reduce, the HIP path of
gloo/math.h:15-73) against the oracle and the reference's golden outputs.
Bit-exact for every dtype; the only relaxation is that a NaN produced by an
fp32/fp64 sum or product may carry a different payload than x86's (both are
NaN) -- selection ops (max/min) and float16 (NaN -> 0x7fff) stay bit-exact."""
import numpy as np
import pytest

from helpers import GOLDEN
from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ALL_DTYPES = [O.INT8, O.UINT8, O.INT32, O.INT64, O.UINT64, O.FLOAT32, O.FLOAT64,
              O.FLOAT16, O.BFLOAT16]
ALL_OPS = [O.SUM, O.PRODUCT, O.MAX, O.MIN]

TORCH_VIEW = {
    O.INT8: torch.int8, O.UINT8: torch.uint8, O.INT32: torch.int32, O.INT64: torch.int64,
    O.UINT64: torch.int64, O.FLOAT32: torch.float32, O.FLOAT64: torch.float64,
    O.FLOAT16: torch.float16, O.BFLOAT16: torch.bfloat16,
}


def to_dev(a, dtype):
    """numpy array -> device tensor of the matching torch dtype (same bits)."""
    if a.size == 0:
        return torch.empty(0, dtype=TORCH_VIEW[dtype], device="cuda")
    t = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy())
    return t.cuda().view(TORCH_VIEW[dtype])


def from_dev(t, dtype):
    if t.numel() == 0:
        return np.zeros(0, dtype=O.NP_DTYPE[dtype])
    return t.cpu().view(torch.uint8).numpy().view(O.NP_DTYPE[dtype])


def gpu_reduce(op, dtype, a, b, inplace=True, c=None, offset=0):
    import ctypes
    import gloo_amd
    from gloo_amd import _lib
    n = a.size
    pad = 64
    A = to_dev(np.concatenate([np.zeros(offset, a.dtype), a, np.zeros(pad, a.dtype)]), dtype)
    B = to_dev(np.concatenate([np.zeros(offset, b.dtype), b, np.zeros(pad, b.dtype)]), dtype)
    es = np.dtype(O.NP_DTYPE[dtype]).itemsize
    pa = A.data_ptr() + offset * es
    pb = B.data_ptr() + offset * es
    if inplace:
        pc, C = pa, A
    else:
        c0 = np.zeros_like(a) if c is None else c
        C = to_dev(np.concatenate([np.zeros(offset, a.dtype), c0, np.zeros(pad, a.dtype)]), dtype)
        pc = C.data_ptr() + offset * es
    stream = torch.cuda.current_stream().cuda_stream
    rc = _lib.lib.glx_reduce(op, dtype, ctypes.c_void_p(pc), ctypes.c_void_p(pa),
                             ctypes.c_void_p(pb), n, ctypes.c_void_p(stream))
    gloo_amd.errors.check(rc, "glx_reduce")
    torch.cuda.synchronize()
    full = from_dev(C, dtype)
    assert np.all(full[offset + n:] == 0), "kernel wrote past the end"
    assert np.all(full[:offset] == 0), "kernel wrote before the start"
    return full[offset:offset + n]


def assert_same(got, exp, dtype, op):
    if dtype in (O.FLOAT32, O.FLOAT64) and op in (O.SUM, O.PRODUCT):
        gn, en = np.isnan(got), np.isnan(exp)
        assert np.array_equal(gn, en), "NaN positions differ"
        got, exp = got[~gn], exp[~en]
    assert np.array_equal(np.ascontiguousarray(got).view(np.uint8),
                          np.ascontiguousarray(exp).view(np.uint8)), \
        "mismatch at %s" % np.nonzero(got != exp)[0][:10]


@pytest.mark.parametrize("dtype", ALL_DTYPES, ids=[O.DTYPE_NAMES[d] for d in ALL_DTYPES])
@pytest.mark.parametrize("op", ALL_OPS, ids=[O.OP_NAMES[o] for o in ALL_OPS])
def test_reduce_vs_oracle(dtype, op):
    for n, off in ((1, 0), (7, 1), (1000, 0), (4099, 3), (65536 + 5, 1), (1 << 20, 0)):
        a = O.fill(dtype, n, 0, seed=11, rank=0)
        b = O.fill(dtype, n, 0, seed=11, rank=1)
        assert_same(gpu_reduce(op, dtype, a, b, offset=off), O.reduce(op, dtype, a, b),
                    dtype, op)
        c = O.fill(dtype, n, 0, seed=11, rank=2)
        assert_same(gpu_reduce(op, dtype, a, b, inplace=False, c=c, offset=off),
                    O.reduce(op, dtype, a, b, inplace=False, c=c), dtype, op)


KATS = np.load(GOLDEN + "/reduce_kats.npz")
KAT_KEYS = sorted({k.rsplit("_", 1)[0] for k in KATS.files if k.endswith("_a")})
DT = {v: k for k, v in O.DTYPE_NAMES.items()}
OPS = {v: k for k, v in O.OP_NAMES.items()}


@pytest.mark.parametrize("key", KAT_KEYS)
def test_reduce_vs_reference_golden(key):
    _, dname, oname = key.split("_")
    dtype, op = DT[dname], OPS[oname]
    a, b = KATS[key + "_a"], KATS[key + "_b"]
    assert_same(gpu_reduce(op, dtype, a, b), KATS[key + "_ab"], dtype, op)
    assert_same(gpu_reduce(op, dtype, b, a), KATS[key + "_ba"], dtype, op)
    assert_same(gpu_reduce(op, dtype, a, b, inplace=False), KATS[key + "_ab0"], dtype, op)
    assert_same(gpu_reduce(op, dtype, b, a, inplace=False), KATS[key + "_ba0"], dtype, op)


def test_f16_rounding_sweep():
    """Every float16 pair class that rounds: a + b over all 65536 a against a
    few b, vs the oracle (conversion + quirk) -- exhaustive over a."""
    a = np.arange(65536, dtype=np.uint16)
    for bv in (0x0000, 0x0001, 0x3c00, 0x1400, 0x7bff, 0x8001, 0xfbff, 0x7e00):
        b = np.full(65536, bv, dtype=np.uint16)
        for op in ALL_OPS:
            assert_same(gpu_reduce(op, O.FLOAT16, a, b), O.reduce(op, O.FLOAT16, a, b),
                        O.FLOAT16, op)


def test_large_fp32_sum_matches_torch():
    """256 MiB fp32 (the cfg2 size): c = a + b equals torch's IEEE add."""
    import gloo_amd
    n = 64 << 20
    g = torch.Generator(device="cuda").manual_seed(3)
    a = torch.rand(n, device="cuda", generator=g) * 2 - 1
    b = torch.rand(n, device="cuda", generator=g) * 2 - 1
    c = torch.empty_like(a)
    gloo_amd.math.sum(c, a, b)
    torch.cuda.synchronize()
    assert torch.equal(c, a + b)
    a0 = a.clone()
    gloo_amd.math.reduce(gloo_amd.ReductionType.MAX, a, a, b)  # in place
    torch.cuda.synchronize()
    assert torch.equal(a, torch.where(a0 < b, b, a0))


def test_segmented_long_streams_match_torch():
    """Streams over 256 MiB go out as equal segments (reduce_kernels.hip
    kSegBytes): 600 MiB fp32 at a 4-byte offset (a scalar head, three
    segments, a scalar tail), out of place and in place -- an element done
    twice in place would show as a + 2b -- the fold of three sources in
    place, and 520 MiB bf16 in place, all equal to torch's IEEE adds."""
    import gloo_amd
    n = (600 << 20) // 4 + 5
    g = torch.Generator(device="cuda").manual_seed(5)
    A = torch.rand(n + 1, device="cuda", generator=g) * 2 - 1
    B = torch.rand(n + 1, device="cuda", generator=g) * 2 - 1
    a, b = A[1:], B[1:]  # 4 bytes past a 16-byte boundary: a scalar head
    c = torch.empty_like(A)[1:]
    gloo_amd.math.sum(c, a, b)
    torch.cuda.synchronize()
    assert torch.equal(c, a + b)
    del c
    a0 = a.clone()
    gloo_amd.math.sum(a, a, b)
    torch.cuda.synchronize()
    assert torch.equal(a, a0 + b)
    # the fold kernel (several local pointers) segments alike: a left fold
    # of three sources into the first, in place
    C = torch.rand(n + 1, device="cuda", generator=g) * 2 - 1
    c = C[1:]
    a.copy_(a0)
    want = (a0 + b) + c
    gloo_amd.math.reduce_n(gloo_amd.ReductionType.SUM, a, [a, b, c])
    torch.cuda.synchronize()
    assert torch.equal(a, want)
    del A, B, C, a, b, c, a0, want
    m = (520 << 20) // 2
    x = (torch.rand(m, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    y = (torch.rand(m, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    want = x + y
    gloo_amd.math.sum(x, x, y)
    torch.cuda.synchronize()
    assert torch.equal(x, want)


def test_reduce_n_left_fold():
    import gloo_amd
    for dtype in (O.FLOAT32, O.FLOAT16, O.INT32):
        n = 10007
        srcs = [O.fill(dtype, n, 0, seed=5, rank=r) for r in range(5)]
        exp = srcs[0]
        for s in srcs[1:]:
            exp = O.reduce(O.SUM, dtype, exp, s)
        ts = [to_dev(s, dtype) for s in srcs]
        gloo_amd.math.reduce_n(gloo_amd.ReductionType.SUM, ts[0], ts)
        torch.cuda.synchronize()
        assert_same(from_dev(ts[0], dtype), exp, dtype, O.SUM)


def test_bf16_against_torch_rounding():
    """bfloat16 has no reference type (parity unpinned against gloo); as an
    independent restatement of the same rule -- widen, op in fp32, round to
    nearest even once -- torch's own fp32 -> bf16 conversion must give the
    kernel's bits for sum and product, and torch.where the operand choice of
    max / min (gloo/math.h:51,66 order), on 1M random values incl. specials."""
    import gloo_amd
    g = torch.Generator(device="cuda").manual_seed(17)
    n = 1 << 20
    a = (torch.randn(n, device="cuda", generator=g) * 64).to(torch.bfloat16)
    b = (torch.randn(n, device="cuda", generator=g) * 64).to(torch.bfloat16)
    special = torch.tensor([0.0, -0.0, float("inf"), -float("inf"), 1e-40, -3e38, 3e38],
                           device="cuda").to(torch.bfloat16)
    a[:special.numel()] = special
    b[:special.numel()] = special.flip(0)
    af, bf = a.float(), b.float()
    exp = {gloo_amd.ReductionType.SUM: (af + bf).to(torch.bfloat16),
           gloo_amd.ReductionType.PRODUCT: (af * bf).to(torch.bfloat16),
           gloo_amd.ReductionType.MAX: torch.where(af < bf, b, a),
           gloo_amd.ReductionType.MIN: torch.where(bf < af, b, a)}
    for op, e in exp.items():
        c = torch.empty_like(a)
        gloo_amd.math.reduce(op, c, a, b)
        torch.cuda.synchronize()
        got, want = c.view(torch.int16), e.view(torch.int16)
        nan = torch.isnan(e.float())
        assert torch.equal(torch.isnan(c.float()), nan)
        assert torch.equal(got[~nan], want[~nan]), op
