"""ctypes bindings for the CPU oracle (oracle/liboracle.so) and, where it was
built, the reference itself (oracle/_ref/libgloo_ref.so).

TEST INFRASTRUCTURE ONLY: the checker, never the thing measured or shipped.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))

# dtype codes shared with include/gloo_amd/glx.h (GLX_*), oracle and ref shim.
INT8, UINT8, INT32, INT64, UINT64, FLOAT32, FLOAT64, FLOAT16, BFLOAT16 = range(9)
SUM, PRODUCT, MAX, MIN = 1, 2, 3, 4

NP_DTYPE = {
    INT8: np.int8, UINT8: np.uint8, INT32: np.int32, INT64: np.int64,
    UINT64: np.uint64, FLOAT32: np.float32, FLOAT64: np.float64,
    FLOAT16: np.uint16, BFLOAT16: np.uint16,  # 16-bit floats carried as raw bits
}
DTYPE_NAMES = {
    INT8: "int8", UINT8: "uint8", INT32: "int32", INT64: "int64",
    UINT64: "uint64", FLOAT32: "float32", FLOAT64: "float64",
    FLOAT16: "float16", BFLOAT16: "bfloat16",
}
OP_NAMES = {SUM: "sum", PRODUCT: "product", MAX: "max", MIN: "min"}

RING_CHUNKED, HALVING_DOUBLING = 0, 1
RING = 9  # gloo::AllreduceRing<T> (the glx.h code GLX_ALGO_RING)
BCUBE = 10  # gloo::AllreduceBcube<T> (GLX_ALGO_BCUBE; groups of `base` ranks)

_lib = None
_ref = None


def _load_oracle():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle.so missing: run `make -C oracle`")
        lib = ctypes.CDLL(path)
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        lib.oracle_reduce.argtypes = [i, i, vp, vp, vp, sz]
        lib.oracle_reduce.restype = i
        lib.oracle_sum_f32.argtypes = [vp, vp, vp, sz]
        lib.oracle_sum_f32.restype = None
        lib.oracle_fill.argtypes = [i, i, ctypes.c_uint64, i, i, i, i, sz, vp]
        lib.oracle_fill.restype = None
        for name in ("oracle_allreduce_ring_chunked", "oracle_allreduce_halving_doubling",
                     "oracle_allreduce_ring"):
            f = getattr(lib, name)
            f.argtypes = [i, i, i, i, i, ctypes.POINTER(vp)]
            f.restype = i
        lib.oracle_allreduce_bcube.argtypes = [i, i, i, i, i, i, ctypes.POINTER(vp)]
        lib.oracle_allreduce_bcube.restype = i
        lib.oracle_allreduce_fn.argtypes = [i, i, i, i, i, i, sz, sz, ctypes.POINTER(vp),
                                            ctypes.POINTER(vp)]
        lib.oracle_allreduce_fn.restype = i
        lib.oracle_f32_to_f16.argtypes = [ctypes.c_float]
        lib.oracle_f32_to_f16.restype = ctypes.c_uint16
        lib.oracle_f16_to_f32.argtypes = [ctypes.c_uint16]
        lib.oracle_f16_to_f32.restype = ctypes.c_float
        for name in ("oracle_f32_to_f16_n", "oracle_f16_to_f32_n", "oracle_f32_to_bf16_n"):
            getattr(lib, name).argtypes = [vp, vp, sz]
            getattr(lib, name).restype = None
        _lib = lib
    return _lib


def ref_available():
    return os.path.exists(os.path.join(_HERE, "_ref", "libgloo_ref.so"))


def _load_ref():
    global _ref
    if _ref is None:
        path = os.path.join(_HERE, "_ref", "libgloo_ref.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/_ref/libgloo_ref.so not built (needs /root/reference)")
        lib = ctypes.CDLL(path)
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        lib.ref_reduce.argtypes = [i, i, vp, vp, vp, sz]
        lib.ref_reduce.restype = i
        lib.ref_allreduce.argtypes = [i, i, i, i, i, i, ctypes.POINTER(vp), i, i,
                                      ctypes.POINTER(ctypes.c_double)]
        lib.ref_allreduce.restype = i
        lib.ref_set_bcube_base.argtypes = [i]
        lib.ref_set_bcube_base.restype = None
        lib.ref_allreduce_fn.argtypes = [i, i, i, i, i, i, sz, sz, ctypes.POINTER(vp),
                                         ctypes.POINTER(vp)]
        lib.ref_allreduce_fn.restype = i
        lib.ref_last_error.restype = ctypes.c_char_p
        lib.ref_reduce_mt.argtypes = [i, i, vp, vp, vp, sz, i, i, ctypes.POINTER(ctypes.c_double)]
        lib.ref_reduce_mt.restype = i
        lib.ref_f32_to_f16.argtypes = [vp, vp, sz]
        lib.ref_f16_to_f32.argtypes = [vp, vp, sz]
        _ref = lib
    return _ref


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def fill(dtype, n, kind=0, seed=1234, rank=0, ptr_index=0, stride=1, val=0):
    """Synthetic input of SURVEY.md 8d (kind 0), the reference stride pattern
    (kind 1, gloo/test/base_test.h:184-191) or a constant (kind 2)."""
    out = np.empty(n, dtype=NP_DTYPE[dtype])
    _load_oracle().oracle_fill(dtype, kind, seed, rank, ptr_index, stride, val, n,
                               _ptr(out))
    return out


def reduce(op, dtype, a, b, use_ref=False, inplace=True, c=None):
    """Elementwise reference semantics (gloo/math.h:15-73).  inplace=True:
    the allreduce form sum(a, b) == sum(a, a, b); otherwise c = op(a, b) into
    `c` (zeros by default, as gloo/test/math_test.cc initialises it).  The
    prior contents of c matter for float16 (see oracle/gloo_oracle.c)."""
    assert a.shape == b.shape
    if inplace:
        c = np.array(a, copy=True)
        a = c
    elif c is None:
        c = np.zeros_like(a)
    else:
        c = np.array(c, copy=True)
    lib = _load_ref() if use_ref else _load_oracle()
    f = lib.ref_reduce if use_ref else lib.oracle_reduce
    rc = f(op, dtype, _ptr(c), _ptr(a), _ptr(b), a.size)
    if rc != 0:
        raise ValueError("reduce rc=%d" % rc)
    return c


def sum_f32(c, a, b):
    """The reference's scalar hot loop, restated (cpu_baseline 'port')."""
    _load_oracle().oracle_sum_f32(_ptr(c), _ptr(a), _ptr(b), a.size)


def allreduce(algo, op, dtype, inputs, use_ref=False, warmup=0, iters=1, base=2):
    """inputs: list (per rank) of lists (per ptr) of 1-D numpy arrays.
    Returns new arrays holding the allreduced result, same nesting.
    algo: RING_CHUNKED, HALVING_DOUBLING, RING (AllreduceRing: each rank's
    own left fold, so float results may differ between ranks) or BCUBE
    (AllreduceBcube with groups of `base` ranks, gloo::Context::base)."""
    P = len(inputs)
    nptrs = len(inputs[0])
    count = inputs[0][0].size
    bufs = [[np.array(x, copy=True) for x in rank] for rank in inputs]
    flat = (ctypes.c_void_p * (P * nptrs))()
    for r in range(P):
        for i in range(nptrs):
            flat[r * nptrs + i] = bufs[r][i].ctypes.data
    if use_ref:
        lib = _load_ref()
        secs = ctypes.c_double(0.0)
        lib.ref_set_bcube_base(int(base))
        rc = lib.ref_allreduce(algo, op, dtype, P, nptrs, count, flat, warmup, iters,
                               ctypes.byref(secs))
        if rc != 0:
            raise RuntimeError("reference allreduce failed rc=%d: %s"
                               % (rc, lib.ref_last_error().decode()))
        allreduce.last_seconds = secs.value
    else:
        lib = _load_oracle()
        if algo == BCUBE:
            rc = lib.oracle_allreduce_bcube(op, dtype, P, nptrs, count, int(base), flat)
        else:
            f = {RING_CHUNKED: lib.oracle_allreduce_ring_chunked,
                 HALVING_DOUBLING: lib.oracle_allreduce_halving_doubling,
                 RING: lib.oracle_allreduce_ring}[algo]
            rc = f(op, dtype, P, nptrs, count, flat)
        if rc != 0:
            raise RuntimeError("oracle allreduce failed rc=%d" % rc)
    return bufs


FN_RING = 1   # AllreduceOptions::Algorithm::RING (gloo/allreduce.h:40)
FN_BCUBE = 2  # AllreduceOptions::Algorithm::BCUBE


def allreduce_fn(algo, op, dtype, inputs, outputs, max_segment_size=0, use_ref=False):
    """gloo::allreduce(opts) over P ranks (gloo/allreduce.cc:97-146).
    inputs: per rank a list (maybe empty) of 1-D arrays; outputs: per rank a
    non-empty list of 1-D arrays holding the outputs' initial contents (they
    are the input when `inputs` is empty).  Returns new output arrays."""
    P = len(outputs)
    nin = len(inputs[0]) if inputs else 0
    nout = len(outputs[0])
    count = outputs[0][0].size
    ins = [[np.array(x, copy=True) for x in (inputs[r] if nin else [])] for r in range(P)]
    outs = [[np.array(x, copy=True) for x in outputs[r]] for r in range(P)]
    fin = (ctypes.c_void_p * max(P * nin, 1))()
    fout = (ctypes.c_void_p * (P * nout))()
    for r in range(P):
        for i in range(nin):
            fin[r * nin + i] = ins[r][i].ctypes.data
        for i in range(nout):
            fout[r * nout + i] = outs[r][i].ctypes.data
    if use_ref:
        lib = _load_ref()
        rc = lib.ref_allreduce_fn(algo, op, dtype, P, nin, nout, count, max_segment_size,
                                  fin, fout)
        if rc != 0:
            raise RuntimeError("reference allreduce failed rc=%d: %s"
                               % (rc, lib.ref_last_error().decode()))
    else:
        rc = _load_oracle().oracle_allreduce_fn(algo, op, dtype, P, nin, nout, count,
                                                max_segment_size, fin, fout)
        if rc != 0:
            raise RuntimeError("oracle allreduce failed rc=%d" % rc)
    return outs


def f32_to_f16(x, use_ref=False):
    """float32 -> float16 bits with cpu_float2half_rn semantics."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty(x.size, dtype=np.uint16)
    if use_ref:
        _load_ref().ref_f32_to_f16(_ptr(x), _ptr(out), x.size)
    else:
        _load_oracle().oracle_f32_to_f16_n(_ptr(x), _ptr(out), x.size)
    return out


def f16_to_f32(h, use_ref=False):
    h = np.ascontiguousarray(h, dtype=np.uint16)
    out = np.empty(h.size, dtype=np.float32)
    if use_ref:
        _load_ref().ref_f16_to_f32(_ptr(h), _ptr(out), h.size)
    else:
        _load_oracle().oracle_f16_to_f32_n(_ptr(h), _ptr(out), h.size)
    return out


def f32_to_bf16(x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty(x.size, dtype=np.uint16)
    _load_oracle().oracle_f32_to_bf16_n(_ptr(x), _ptr(out), x.size)
    return out
