"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Runs liuxiaotiao/gloo's own code -- gloo/math.h, gloo/types.h and
AllreduceRingChunked / AllreduceHalvingDoubling over its tcp transport on
loopback, P thread-ranks sharing a HashStore exactly like
gloo/test/base_test.h:91-166 -- through oracle/_ref/libgloo_ref.so, which
oracle/Makefile compiles from the sources under /root/reference.  Only
inputs and outputs are stored (data, not source).

Inputs are regenerated in the tests from (dtype, kind, seed, rank, ptr) by
oracle.fill(); each fixture stores a checksum of its inputs so generator
drift is caught.

    make -C oracle all ref && python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402

SEED = 1234


def sha(arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).view(np.uint8).tobytes())
    return h.hexdigest()


def edge_values(dtype):
    """Special values the reference's semantics must preserve."""
    if dtype == O.FLOAT32:
        v = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45,
                      1.17549435e-38, 3.4028235e38, -3.4028235e38, 0.1, 1e30, -2.5],
                     dtype=np.float32)
        return v
    if dtype == O.FLOAT64:
        return np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 5e-324,
                         1.7976931348623157e308, 0.1, -2.5], dtype=np.float64)
    if dtype == O.FLOAT16:
        return np.array([0x0000, 0x8000, 0x3c00, 0xbc00, 0x7c00, 0xfc00, 0x7e00, 0x7fff,
                         0xfe01, 0x0001, 0x8001, 0x03ff, 0x0400, 0x7bff, 0xfbff, 0x3555],
                        dtype=np.uint16)
    if dtype in (O.INT8, O.UINT8, O.INT32, O.INT64, O.UINT64):
        info = np.iinfo(O.NP_DTYPE[dtype])
        return np.array([0, 1, info.max, info.min, info.max - 1, 7, 3],
                        dtype=O.NP_DTYPE[dtype])
    raise ValueError(dtype)


def make_reduce():
    """gloo/math.h ops: seeded + edge-value cross products, both orders."""
    out = {}
    meta = []
    for dtype in (O.INT8, O.UINT8, O.INT32, O.INT64, O.UINT64, O.FLOAT32, O.FLOAT64,
                  O.FLOAT16):
        n = 1000
        a = O.fill(dtype, n, 0, seed=SEED, rank=0)
        b = O.fill(dtype, n, 0, seed=SEED, rank=1)
        e = edge_values(dtype)
        ea = np.repeat(e, len(e))
        eb = np.tile(e, len(e))
        A = np.concatenate([a, ea])
        B = np.concatenate([b, eb])
        if dtype == O.FLOAT16:
            # hit the float16 assignment quirk: b = f2h((float)a.x), a < b
            qa = np.array([0x0001, 0x0100, 0x3c00, 0x1234, 0x2000], dtype=np.uint16)
            qb = O.f32_to_f16(qa.astype(np.float32), use_ref=True)
            A = np.concatenate([A, qa, qb])
            B = np.concatenate([B, qb, qa])
        for op in (O.SUM, O.PRODUCT, O.MAX, O.MIN):
            key = "reduce_%s_%s" % (O.DTYPE_NAMES[dtype], O.OP_NAMES[op])
            out[key + "_a"] = A
            out[key + "_b"] = B
            # in place (the allreduce form) and into a zeroed c, both orders
            out[key + "_ab"] = O.reduce(op, dtype, A, B, use_ref=True)
            out[key + "_ba"] = O.reduce(op, dtype, B, A, use_ref=True)
            out[key + "_ab0"] = O.reduce(op, dtype, A, B, use_ref=True, inplace=False)
            out[key + "_ba0"] = O.reduce(op, dtype, B, A, use_ref=True, inplace=False)
            meta.append(key)
    np.savez_compressed(os.path.join(HERE, "reduce_kats.npz"), **out)
    return meta


def make_f16_conversions():
    """cpu_float2half_rn over a strided sweep of all float bit patterns plus
    every float that is exactly a half or a half midpoint."""
    rng = np.random.default_rng(SEED)
    stride = np.arange(0, 2**32, 65537, dtype=np.uint64).astype(np.uint32)
    halves = np.arange(0, 2**16, dtype=np.uint32)
    # exact halves and midpoints (as float bits) -- the RNE tie cases
    h16 = halves.astype(np.uint16)
    hf = np.empty(halves.size, dtype=np.float32)
    O._load_ref().ref_f16_to_f32(O._ptr(h16), O._ptr(hf), halves.size)
    hb = hf.view(np.uint32)
    mids = hb[np.isfinite(hf)] + np.uint32(1 << 12)  # not exact midpoints for all, plus
    near = np.concatenate([hb, hb + 1, hb - 1, mids, mids + 1, mids - 1])
    rnd = rng.integers(0, 2**32, size=50000, dtype=np.uint64).astype(np.uint32)
    bits = np.unique(np.concatenate([stride, near.astype(np.uint32), rnd]))
    f = bits.view(np.float32)
    h = O.f32_to_f16(f, use_ref=True)
    np.savez_compressed(os.path.join(HERE, "f16_conversions.npz"), f32_bits=bits, f16=h,
                        half_bits=h16, half_to_f32_bits=hf.view(np.uint32))


ALLREDUCE_CASES = []
for algo in (O.RING_CHUNKED, O.HALVING_DOUBLING):
    for P in (1, 2, 3, 4, 5, 7, 8):
        for N in (1, 255, 256, 1024, 4099, 100003):
            ALLREDUCE_CASES.append((algo, P, N, O.FLOAT32, O.SUM, 1, 0))
    for P in (2, 4, 8):
        ALLREDUCE_CASES.append((algo, P, 4099, O.INT32, O.SUM, 1, 0))
        ALLREDUCE_CASES.append((algo, P, 4099, O.FLOAT16, O.SUM, 1, 0))
        ALLREDUCE_CASES.append((algo, P, 1000, O.FLOAT32, O.MAX, 1, 0))
        ALLREDUCE_CASES.append((algo, P, 1000, O.FLOAT32, O.MIN, 2, 0))
        ALLREDUCE_CASES.append((algo, P, 1000, O.FLOAT32, O.PRODUCT, 1, 0))
    # the reference tests' own integer-valued patterns
    for P in (3, 6):
        ALLREDUCE_CASES.append((algo, P, 10000, O.FLOAT32, O.SUM, 1, 2))  # value = rank
        ALLREDUCE_CASES.append((algo, P, 1000, O.FLOAT32, O.SUM, 2, 1))   # stride pattern
        ALLREDUCE_CASES.append((algo, P, 1024, O.FLOAT16, O.SUM, 1, 2))


def case_inputs(P, N, dtype, nptrs, kind):
    ins = []
    for r in range(P):
        row = []
        for i in range(nptrs):
            if kind == 0:
                row.append(O.fill(dtype, N, 0, seed=SEED, rank=r, ptr_index=i))
            elif kind == 1:  # base_test.h:184-191
                stride = P * nptrs
                row.append(O.fill(dtype, N, 1, stride=stride, val=r * nptrs + i))
            else:  # allreduce_test.cc:156-158
                row.append(O.fill(dtype, N, 2, val=r))
        ins.append(row)
    return ins


def case_name(c):
    algo, P, N, dtype, op, nptrs, kind = c
    return "%s_P%d_N%d_%s_%s_p%d_k%d" % (
        "ring" if algo == O.RING_CHUNKED else "hd", P, N, O.DTYPE_NAMES[dtype],
        O.OP_NAMES[op], nptrs, kind)


def make_allreduce():
    out = {}
    index = []
    for c in ALLREDUCE_CASES:
        algo, P, N, dtype, op, nptrs, kind = c
        ins = case_inputs(P, N, dtype, nptrs, kind)
        res = O.allreduce(algo, op, dtype, ins, use_ref=True)
        first = res[0][0]
        for r in range(P):
            for i in range(nptrs):
                assert np.array_equal(res[r][i].view(np.uint8), first.view(np.uint8)), \
                    "reference ranks disagree in %s" % case_name(c)
        name = case_name(c)
        rec = {"name": name, "algo": algo, "P": P, "N": N, "dtype": dtype, "op": op,
               "nptrs": nptrs, "kind": kind, "seed": SEED,
               "input_sha256": sha([x for row in ins for x in row]),
               "output_sha256": sha([first])}
        if N <= 4099:
            out[name] = first
        else:  # large: store a sample + checksum
            idx = np.linspace(0, N - 1, 257).astype(np.int64)
            out[name + "_idx"] = idx
            out[name + "_sample"] = first[idx]
        index.append(rec)
        print(name, flush=True)
    np.savez_compressed(os.path.join(HERE, "allreduce_golden.npz"), **out)
    with open(os.path.join(HERE, "allreduce_golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "source": "oracle/_ref/libgloo_ref.so (reference compiled from "
                             "/root/reference by oracle/Makefile)",
                   "cases": index}, f, indent=1)


# ---- gloo::AllreduceRing<T> (gloo/allreduce_ring.h) ----------------------
# Each rank's result is its own left fold (x[r] op x[r-1] op ...), so float
# outputs differ between ranks: every rank's output is recorded.  N = 0 is a
# no-op (run() returns first, :72-74); the compiled reference's P >= 3 runs of
# it end in a teardown race of its tcp pairs, so it is not generated here.
RING_CASES = []
for _P in range(1, 16):  # the reference test's own grid (allreduce_test.cc:241-249)
    for _N in (4, 100, 1000, 10000):
        RING_CASES.append((_P, _N, O.FLOAT32, O.SUM, 1, 2))  # value = rank (:156-158)
for _P in (2, 3, 5, 8):
    for _N in (1, 1000, 4099, 100003):
        RING_CASES.append((_P, _N, O.FLOAT32, O.SUM, 1, 0))
for _P in (3, 8):
    RING_CASES.append((_P, 4099, O.FLOAT16, O.SUM, 1, 0))
    RING_CASES.append((_P, 1000, O.FLOAT32, O.MAX, 1, 0))
    RING_CASES.append((_P, 1000, O.FLOAT32, O.PRODUCT, 1, 0))
RING_CASES.append((4, 4099, O.INT32, O.SUM, 1, 0))
RING_CASES.append((4, 1000, O.FLOAT32, O.MIN, 2, 0))
RING_CASES.append((2, 4099, O.FLOAT32, O.SUM, 3, 0))
RING_CASES.append((5, 1000, O.FLOAT32, O.SUM, 2, 1))  # stride pattern (base_test.h:184-191)


def ring_case_name(c):
    P, N, dtype, op, nptrs, kind = c
    return "allreduce_ring_P%d_N%d_%s_%s_p%d_k%d" % (P, N, O.DTYPE_NAMES[dtype],
                                                     O.OP_NAMES[op], nptrs, kind)


def make_ring():
    out = {}
    index = []
    for c in RING_CASES:
        P, N, dtype, op, nptrs, kind = c
        ins = case_inputs(P, N, dtype, nptrs, kind)
        res = O.allreduce(O.RING, op, dtype, ins, use_ref=True)
        name = ring_case_name(c)
        rec = {"name": name, "algo": O.RING, "P": P, "N": N, "dtype": dtype, "op": op,
               "nptrs": nptrs, "kind": kind, "seed": SEED,
               "input_sha256": sha([x for row in ins for x in row]),
               "output_sha256": [sha(row) for row in res]}
        for r in range(P):
            for i in range(1, nptrs):  # the local broadcast
                assert np.array_equal(res[r][i].view(np.uint8), res[r][0].view(np.uint8))
            if N <= 4099:
                out["%s_r%d" % (name, r)] = res[r][0]
        index.append(rec)
        print(name, flush=True)
    np.savez_compressed(os.path.join(HERE, "allreduce_ring_golden.npz"), **out)
    with open(os.path.join(HERE, "allreduce_ring_golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py ring",
                   "source": "oracle/_ref/libgloo_ref.so (gloo::AllreduceRing<T> compiled "
                             "from /root/reference by oracle/Makefile), P thread-ranks over "
                             "TCP loopback",
                   "cases": index}, f, indent=1)


# ---- gloo::AllreduceBcube<T> (gloo/allreduce_bcube.h) --------------------
# Groups of gloo::Context::base ranks.  The reference test's grid
# (allreduce_test.cc:271-299: base 2 at P = 1, 2, 4, 8, 16; base 3 at 1, 3, 9,
# 27; base 4 at 1, 4, 16; N = 1, 64, 1000 -- 0 is a no-op), plus seeded
# order-sensitive inputs at other P (its groups need not be full).  With fewer
# elements than group members the reference's ranges wrap and ranks can end
# with differently ordered sums: every rank's digest is recorded.
BCUBE_CASES = []
for _b, _Ps in ((2, (1, 2, 4, 8, 16)), (3, (1, 3, 9, 27)), (4, (1, 4, 16))):
    for _P in _Ps:
        for _N in (1, 64, 1000):
            BCUBE_CASES.append((_b, _P, _N, O.FLOAT32, O.SUM, 1, 2))
for _b, _Ps in ((2, (3, 5, 8)), (3, (4, 9)), (4, (6,))):
    for _P in _Ps:
        for _N in (3, 1000, 100003):
            BCUBE_CASES.append((_b, _P, _N, O.FLOAT32, O.SUM, 1, 0))
for _b, _P in ((2, 8), (3, 9)):
    BCUBE_CASES.append((_b, _P, 4099, O.FLOAT16, O.SUM, 1, 0))
    BCUBE_CASES.append((_b, _P, 4099, O.INT32, O.MAX, 1, 0))
    BCUBE_CASES.append((_b, _P, 1000, O.FLOAT32, O.PRODUCT, 2, 0))
BCUBE_CASES.append((2, 4, 1000, O.FLOAT32, O.MIN, 3, 1))


def bcube_case_name(c):
    base, P, N, dtype, op, nptrs, kind = c
    return "allreduce_bcube_b%d_P%d_N%d_%s_%s_p%d_k%d" % (base, P, N, O.DTYPE_NAMES[dtype],
                                                          O.OP_NAMES[op], nptrs, kind)


def make_bcube():
    out = {}
    index = []
    for c in BCUBE_CASES:
        base, P, N, dtype, op, nptrs, kind = c
        ins = case_inputs(P, N, dtype, nptrs, kind)
        res = O.allreduce(O.BCUBE, op, dtype, ins, use_ref=True, base=base)
        name = bcube_case_name(c)
        rec = {"name": name, "algo": O.BCUBE, "base": base, "P": P, "N": N, "dtype": dtype,
               "op": op, "nptrs": nptrs, "kind": kind, "seed": SEED,
               "input_sha256": sha([x for row in ins for x in row]),
               "output_sha256": [sha(row) for row in res]}
        for r in range(P):
            if N <= 4099:
                out["%s_r%d" % (name, r)] = res[r][0]
        index.append(rec)
        print(name, flush=True)
    np.savez_compressed(os.path.join(HERE, "allreduce_bcube_golden.npz"), **out)
    with open(os.path.join(HERE, "allreduce_bcube_golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py bcube",
                   "source": "oracle/_ref/libgloo_ref.so (gloo::AllreduceBcube<T> compiled "
                             "from /root/reference by oracle/Makefile), P thread-ranks over "
                             "TCP loopback, gloo::Context::base = base",
                   "cases": index}, f, indent=1)


# ---- gloo::allreduce(AllreduceOptions) (gloo/allreduce.cc) ----------------
# (algo, P, N, dtype, op, nin, nout, max_seg, kind, out_init)
#   kind      0 seeded, 1 stride pattern (base_test.h:184-191)
#   out_init  "pattern": the outputs hold the data (in place, no inputs);
#             "zero": outputs cleared (allreduce_test.cc:325-327);
#             "seeded": outputs hold other seeded data (exposes float16's
#             assignment reading the destination, gloo/types.h)
FN_CASES = []
for _algo in (O.FN_RING, O.FN_BCUBE):
    # the reference's AllreduceNewTest grid (allreduce_test.cc:306-378), uint64 sum,
    # maxSegmentSize 128
    for _P in (1, 2, 4, 7):
        for _np in (1, 2, 3):
            for _N in (0, 1, 10, 100, 1000, 10000):
                FN_CASES.append((_algo, _P, _N, O.UINT64, O.SUM, 0, _np, 128, 1, "pattern"))
                FN_CASES.append((_algo, _P, _N, O.UINT64, O.SUM, _np, _np, 128, 1, "zero"))
    # seeded data, rounding-sensitive types and every op
    for _P in (2, 3, 5, 8):
        for _N, _ms in ((1000, 0), (4099, 128), (100003, 0), (100003, 4096)):
            FN_CASES.append((_algo, _P, _N, O.FLOAT32, O.SUM, 0, 1, _ms, 0, "pattern"))
        FN_CASES.append((_algo, _P, 4099, O.INT32, O.SUM, 2, 1, 256, 0, "seeded"))
        FN_CASES.append((_algo, _P, 4099, O.FLOAT16, O.SUM, 2, 2, 256, 0, "seeded"))
        FN_CASES.append((_algo, _P, 4099, O.FLOAT16, O.MAX, 3, 1, 0, 0, "seeded"))
        FN_CASES.append((_algo, _P, 2048, O.FLOAT16, O.MIN, 0, 2, 0, 0, "pattern"))
        FN_CASES.append((_algo, _P, 1000, O.FLOAT32, O.MAX, 1, 1, 0, 0, "seeded"))
        FN_CASES.append((_algo, _P, 1000, O.FLOAT64, O.PRODUCT, 0, 1, 0, 0, "pattern"))


def fn_case_buffers(c):
    """(inputs, outputs) per rank of a FN_CASES entry, as the tests rebuild them."""
    algo, P, N, dtype, op, nin, nout, ms, kind, out_init = c
    if out_init == "pattern":
        data = case_inputs(P, N, dtype, nout, kind)
        return [[] for _ in range(P)], data
    ins = case_inputs(P, N, dtype, nin, kind)
    if out_init == "zero":
        outs = [[np.zeros(N, dtype=O.NP_DTYPE[dtype]) for _ in range(nout)] for _ in range(P)]
    else:
        outs = [[O.fill(dtype, N, 0, seed=SEED + 1, rank=r, ptr_index=i) for i in range(nout)]
                for r in range(P)]
    return ins, outs


def fn_case_name(c):
    algo, P, N, dtype, op, nin, nout, ms, kind, out_init = c
    return "%s_P%d_N%d_%s_%s_in%d_out%d_seg%d_k%d_%s" % (
        "ring" if algo == O.FN_RING else "bcube", P, N, O.DTYPE_NAMES[dtype],
        O.OP_NAMES[op], nin, nout, ms, kind, out_init)


def make_allreduce_fn():
    out = {}
    index = []
    for c in FN_CASES:
        algo, P, N, dtype, op, nin, nout, ms, kind, out_init = c
        ins, outs = fn_case_buffers(c)
        res = O.allreduce_fn(algo, op, dtype, ins, outs, ms, use_ref=True)
        first = res[0][0]
        for r in range(P):
            for i in range(nout):
                assert np.array_equal(res[r][i].view(np.uint8), first.view(np.uint8)), \
                    "reference ranks disagree in %s" % fn_case_name(c)
        name = fn_case_name(c)
        rec = {"name": name, "algo": algo, "P": P, "N": N, "dtype": dtype, "op": op,
               "nin": nin, "nout": nout, "max_segment_size": ms, "kind": kind,
               "out_init": out_init, "seed": SEED,
               "input_sha256": sha([x for row in ins + outs for x in row]),
               "output_sha256": sha([first])}
        if N <= 4099:
            out[name] = first
        else:
            idx = np.linspace(0, N - 1, 257).astype(np.int64)
            out[name + "_idx"] = idx
            out[name + "_sample"] = first[idx]
        index.append(rec)
    np.savez_compressed(os.path.join(HERE, "allreduce_fn_golden.npz"), **out)
    with open(os.path.join(HERE, "allreduce_fn_golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (make_allreduce_fn)",
                   "source": "gloo::allreduce(AllreduceOptions) of oracle/_ref/libgloo_ref.so "
                             "(reference compiled from /root/reference by oracle/Makefile)",
                   "cases": index}, f, indent=1)
    print("allreduce_fn: %d cases" % len(index))


# ---- gloo::allreduce(opts) with a caller's reduction function --------------
# oracle/ref_harness.cc's custom Funcs over 32-bit words: 100 = a | b, 101 =
# 3a + b (mod 2^32; neither commutative nor associative, so the output bits
# pin every call's order and operands).  The product runs them on host
# buffers (glx_allreduce_host_fn).
CUSTOM_OR, CUSTOM_3A_PLUS_B = 100, 101
CUSTOM_CASES = []
for _algo in (O.FN_RING, O.FN_BCUBE):
    for _P in (1, 2, 3, 4, 5, 8):
        for _N, _nin, _nout, _ms in ((1, 0, 1, 0), (17, 1, 1, 0), (1000, 2, 1, 0),
                                     (4099, 0, 1, 1024), (4099, 3, 2, 0), (65537, 0, 3, 4096)):
            for _op in (CUSTOM_OR, CUSTOM_3A_PLUS_B):
                CUSTOM_CASES.append((_algo, _P, _N, _op, _nin, _nout, _ms))


def custom_case_buffers(c):
    """(inputs, outputs) per rank of a CUSTOM_CASES entry (int32 words): the
    tests rebuild them with the same calls."""
    algo, P, N, op, nin, nout, ms = c
    ins = [[O.fill(O.INT32, N, 0, seed=SEED + 7, rank=r, ptr_index=i) for i in range(nin)]
           for r in range(P)]
    outs = [[O.fill(O.INT32, N, 0, seed=SEED + 8, rank=r, ptr_index=i) for i in range(nout)]
            for r in range(P)]
    return ins, outs


def custom_case_name(c):
    algo, P, N, op, nin, nout, ms = c
    return "%s_P%d_N%d_%s_in%d_out%d_seg%d" % (
        "ring" if algo == O.FN_RING else "bcube", P, N,
        {CUSTOM_OR: "or", CUSTOM_3A_PLUS_B: "3a_plus_b"}[op], nin, nout, ms)


def make_allreduce_custom():
    out = {}
    index = []
    for c in CUSTOM_CASES:
        algo, P, N, op, nin, nout, ms = c
        ins, outs = custom_case_buffers(c)
        res = O.allreduce_fn(algo, op, O.INT32, ins, outs, ms, use_ref=True)
        first = res[0][0]
        for r in range(P):
            for i in range(nout):
                assert np.array_equal(res[r][i], first), \
                    "reference ranks disagree in %s" % custom_case_name(c)
        name = custom_case_name(c)
        index.append({"name": name, "algo": algo, "P": P, "N": N, "op": op, "nin": nin,
                      "nout": nout, "max_segment_size": ms, "seed": SEED,
                      "input_sha256": sha([x for row in ins + outs for x in row]),
                      "output_sha256": sha([first])})
        if N <= 4099:
            out[name] = first
        else:  # the digest pins it; a sample says where a mismatch starts
            idx = np.linspace(0, N - 1, 257).astype(np.int64)
            out[name + "_idx"] = idx
            out[name + "_sample"] = first[idx]
    np.savez_compressed(os.path.join(HERE, "allreduce_custom_golden.npz"), **out)
    with open(os.path.join(HERE, "allreduce_custom_golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (make_allreduce_custom)",
                   "source": "gloo::allreduce(AllreduceOptions) with oracle/ref_harness.cc's "
                             "custom Funcs (100: a | b, 101: 3a + b mod 2^32 on 32-bit words) "
                             "of oracle/_ref/libgloo_ref.so (reference compiled from "
                             "/root/reference by oracle/Makefile)",
                   "cases": index}, f, indent=1)
    print("allreduce_custom: %d cases" % len(index))


# ---- the class algorithms with a CUSTOM ReductionFunction<T> ---------------
# gloo::AllreduceRingChunked<T> / AllreduceHalvingDoubling<T> constructed with
# ReductionFunction<T>(CUSTOM, fn), fn(T* x, const T* y, n): x = f(x, y)
# (gloo/algorithm.h:58-83) -- oracle/ref_harness.cc's classOr / class3aPlusB
# over int32 words.  Host buffers; every pointer of every rank ends equal.
CLASS_CUSTOM_CASES = []
for _algo in (O.RING_CHUNKED, O.HALVING_DOUBLING):
    for _op in (CUSTOM_OR, CUSTOM_3A_PLUS_B):
        for _P in (1, 2, 3, 4, 5, 8):
            for _N in (7, 1000, 4099):
                for _np in (1, 2):
                    CLASS_CUSTOM_CASES.append((_algo, _P, _N, _op, _np))
        for _P in (3, 8):
            CLASS_CUSTOM_CASES.append((_algo, _P, 100003, _op, 1))
        CLASS_CUSTOM_CASES.append((_algo, 6, 4099, _op, 3))


def class_custom_case_name(c):
    algo, P, N, op, nptrs = c
    return "%s_P%d_N%d_%s_p%d" % ("ring" if algo == O.RING_CHUNKED else "hd", P, N,
                                  {CUSTOM_OR: "or", CUSTOM_3A_PLUS_B: "3a_plus_b"}[op], nptrs)


def make_allreduce_class_custom():
    out = {}
    index = []
    for c in CLASS_CUSTOM_CASES:
        algo, P, N, op, nptrs = c
        ins = case_inputs(P, N, O.INT32, nptrs, 0)
        res = O.allreduce(algo, op, O.INT32, ins, use_ref=True)
        first = res[0][0]
        for r in range(P):
            for i in range(nptrs):
                assert np.array_equal(res[r][i], first), \
                    "reference ranks disagree in %s" % class_custom_case_name(c)
        name = class_custom_case_name(c)
        index.append({"name": name, "algo": algo, "P": P, "N": N, "op": op, "nptrs": nptrs,
                      "seed": SEED, "input_sha256": sha([x for row in ins for x in row]),
                      "output_sha256": sha([first])})
        if N <= 4099:
            out[name] = first
        else:
            idx = np.linspace(0, N - 1, 257).astype(np.int64)
            out[name + "_idx"] = idx
            out[name + "_sample"] = first[idx]
    np.savez_compressed(os.path.join(HERE, "allreduce_class_custom_golden.npz"), **out)
    with open(os.path.join(HERE, "allreduce_class_custom_golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (make_allreduce_class_custom)",
                   "source": "gloo::AllreduceRingChunked<int32_t> / AllreduceHalvingDoubling"
                             "<int32_t> with oracle/ref_harness.cc's CUSTOM ReductionFunctions "
                             "(100: x | y, 101: 3x + y mod 2^32) of oracle/_ref/libgloo_ref.so "
                             "(reference compiled from /root/reference by oracle/Makefile)",
                   "cases": index}, f, indent=1)
    print("allreduce_class_custom: %d cases" % len(index))


# ---- BASELINE.json configs at full size (digests, not arrays) -------------
# cfg3: ring_chunked fp32, 8 ranks, the 1K..16M element sweep;
# cfg4: halving_doubling fp32, 8 ranks, 256 MiB per rank;
# cfg5: ring_chunked fp16, 8 ranks, 1 GiB per rank (bf16: the oracle's
#       restatement -- the reference has no bfloat16, parity unpinned).
# Inputs are O.fill(dtype, N, seed=SEED, rank=r); the tests
# regenerate them on each rank and compare SHA-256 digests.
SCALE_CASES = [(O.RING_CHUNKED, 8, 1 << k, O.FLOAT32) for k in range(10, 25, 2)]
# cfg5 is 1 GiB per rank: 2^29 16-bit elements (536,870,912;
# the reference's `int count` holds it, gloo/allreduce_ring_chunked.h:239-240)
CFG5_CASES = [(O.RING_CHUNKED, 8, 1 << 29, O.FLOAT16),
              (O.RING_CHUNKED, 8, 1 << 29, O.BFLOAT16)]
SCALE_CASES += [(O.HALVING_DOUBLING, 8, 1 << 26, O.FLOAT32)] + CFG5_CASES


def scale_case_name(c):
    algo, P, N, dtype = c
    return "%s_P%d_N%d_%s_sum" % ("ring" if algo == O.RING_CHUNKED else "hd", P, N,
                                  O.DTYPE_NAMES[dtype])


def make_scale(only=None):
    """Every BASELINE-scale case, or (only = a list of cases) just those,
    replacing the same-named or same-(algo, P, dtype) entries of the existing
    file (cfg5 alone: `make_golden.py scale5`, ~40 GiB of RAM)."""
    path = os.path.join(HERE, "scale_golden.json")
    cases = []
    todo = SCALE_CASES if only is None else only
    for c in todo:
        algo, P, N, dtype = c
        ins = [[O.fill(dtype, N, 0, seed=SEED, rank=r)] for r in range(P)]
        pinned = dtype != O.BFLOAT16
        res = O.allreduce(algo, O.SUM, dtype, ins, use_ref=pinned)
        first = res[0][0]
        for r in range(P):
            assert np.array_equal(res[r][0].view(np.uint8), first.view(np.uint8)), \
                "ranks disagree in %s" % scale_case_name(c)
        idx = np.linspace(0, N - 1, 65).astype(np.int64)
        cases.append({
            "name": scale_case_name(c), "algo": algo, "P": P, "N": N, "dtype": dtype,
            "op": O.SUM, "seed": SEED,
            "source": "reference" if pinned else "oracle restatement (parity unpinned)",
            "input_sha256": [sha([ins[r][0]]) for r in range(P)],
            "output_sha256": sha([first]),
            "sample_idx": idx.tolist(),
            "sample": [int(v) for v in first.view(np.uint32 if first.itemsize == 4
                                                  else np.uint16)[idx]],
        })
        print(cases[-1]["name"], cases[-1]["output_sha256"][:16], flush=True)
        del ins, res, first
    if only is not None:
        with open(path) as f:
            old = json.load(f)["cases"]
        keys = {(c["algo"], c["P"], c["dtype"]) for c in cases}
        cases = [c for c in old if (c["algo"], c["P"], c["dtype"]) not in keys] + cases
    with open(path, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (make_scale)",
                   "source": "oracle/_ref/libgloo_ref.so (the reference compiled from "
                             "/root/reference by oracle/Makefile), P thread-ranks over "
                             "TCP loopback; bfloat16 from oracle/liboracle.so",
                   "sample_bits": "raw element bits at sample_idx",
                   "cases": cases}, f, indent=1)


# The N > 1 bench workloads (configs[2] / configs[3] at the driver's node
# sizes: 256 MiB fp32 per rank at 2, 4 and 8 ranks), so bench.py can check
# the output of every timed candidate against the reference's own digest.
# The inputs are SURVEY 8d's synthetic values (oracle_fill kind 0, seed 1234,
# rank r), which bench.py regenerates on the device.
BENCH_CASES = [(a, P, 1 << 26, O.FLOAT32) for a in (O.RING_CHUNKED, O.HALVING_DOUBLING)
               for P in (2, 4, 8)]


def make_bench():
    path = os.path.join(HERE, "bench_golden.json")
    cases = []
    for c in BENCH_CASES:
        algo, P, N, dtype = c
        ins = [[O.fill(dtype, N, 0, seed=SEED, rank=r)] for r in range(P)]
        res = O.allreduce(algo, O.SUM, dtype, ins, use_ref=True)
        first = res[0][0]
        for r in range(P):
            assert np.array_equal(res[r][0].view(np.uint8), first.view(np.uint8))
        cases.append({"name": scale_case_name(c), "algo": algo, "P": P, "N": N,
                      "dtype": dtype, "op": O.SUM, "seed": SEED, "source": "reference",
                      "input_sha256": [sha([ins[r][0]]) for r in range(P)],
                      "output_sha256": sha([first])})
        print(cases[-1]["name"], cases[-1]["output_sha256"][:16], flush=True)
        del ins, res, first
    with open(path, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py bench",
                   "source": "oracle/_ref/libgloo_ref.so (the reference compiled from "
                             "/root/reference by oracle/Makefile), P thread-ranks over "
                             "TCP loopback",
                   "inputs": "oracle_fill kind 0 (SURVEY 8d: splitmix64 of seed ^ rank<<40 ^ "
                             "i, ((h>>40) - 2^23) / 2^23), seed 1234; bench.py regenerates "
                             "them on the device and checks their digests too",
                   "cases": cases}, f, indent=1)


if __name__ == "__main__":
    if not O.ref_available():
        sys.exit("oracle/_ref/libgloo_ref.so missing: make -C oracle ref")
    which = sys.argv[1:] or ["reduce", "f16", "allreduce", "allreduce_fn", "ring", "bcube",
                             "custom", "class_custom"]
    if "reduce" in which:
        make_reduce()
    if "f16" in which:
        make_f16_conversions()
    if "allreduce" in which:
        make_allreduce()
    if "allreduce_fn" in which:
        make_allreduce_fn()
    if "ring" in which:
        make_ring()
    if "bcube" in which:
        make_bcube()
    if "custom" in which:
        make_allreduce_custom()
    if "class_custom" in which:
        make_allreduce_class_custom()
    if "scale" in which:  # not in the default set: minutes and ~40 GiB of RAM
        make_scale()
    if "bench" in which:  # bench.py's N > 1 workloads (256 MiB fp32, P = 2, 4, 8)
        make_bench()
    if "scale5" in which:  # cfg5 alone (1 GiB per rank, 8 ranks)
        make_scale(CFG5_CASES)
    print("done")
