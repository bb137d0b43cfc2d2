"""Device elementwise reductions: the hot loop of the allreduce path.

gloo::sum/product/max/min<T>(c, a, b, n) (gloo/math.h:15-73) as HIP kernels
through glx_reduce.  Reference CPU semantics, bit for bit.
"""
import builtins
import ctypes

from . import _lib
from .algorithms import ReductionType, _stream_ptr, torch_dtype_code
from .errors import check

lib = _lib.lib


def reduce(op, c, a, b, n=None, stream=None):
    """c[:n] = op(a[:n], b[:n]) on the device (c may alias a or b).  op is a
    ReductionType value; tensors share dtype and device.  Enqueued on `stream`
    (torch.cuda.Stream or raw hipStream_t) or torch's current stream."""
    dt = torch_dtype_code(c)
    if torch_dtype_code(a) != dt or torch_dtype_code(b) != dt:
        raise TypeError("dtype mismatch")
    if n is None:
        n = builtins.min(c.numel(), a.numel(), b.numel())
    if n > builtins.min(c.numel(), a.numel(), b.numel()):
        raise ValueError("n exceeds a buffer")
    if stream is None:
        import torch
        stream = torch.cuda.current_stream(c.device)
    check(lib.glx_reduce(int(op), dt, c.data_ptr(), a.data_ptr(), b.data_ptr(), int(n),
                         _stream_ptr(stream)), "reduce")
    return c


def reduce_n(op, dst, srcs, n=None, stream=None):
    """dst = left fold of op over srcs (2..8 tensors), one pass."""
    dt = torch_dtype_code(dst)
    if n is None:
        n = builtins.min([dst.numel()] + [s.numel() for s in srcs])
    if stream is None:
        import torch
        stream = torch.cuda.current_stream(dst.device)
    arr = (ctypes.c_void_p * len(srcs))(*[s.data_ptr() for s in srcs])
    check(lib.glx_reduce_n(int(op), dt, dst.data_ptr(), arr, len(srcs), int(n),
                           _stream_ptr(stream)), "reduce_n")
    return dst


def sum(c, a, b, **kw):  # noqa: A001 - gloo's name
    return reduce(ReductionType.SUM, c, a, b, **kw)


def product(c, a, b, **kw):
    return reduce(ReductionType.PRODUCT, c, a, b, **kw)


def max(c, a, b, **kw):  # noqa: A001
    return reduce(ReductionType.MAX, c, a, b, **kw)


def min(c, a, b, **kw):  # noqa: A001
    return reduce(ReductionType.MIN, c, a, b, **kw)


def host_reduce_n(op, dtype, dst, srcs):
    """dst = left fold of op over srcs on HOST memory (numpy arrays of the
    dtype's storage type; dst may be srcs[0]): the local reduce the
    algorithms do on the host for multi-pointer host buffers below
    kOnDeviceThreshold (gloo/algorithm.cc:16).  Same bits as the kernels."""
    n = builtins.min([dst.size] + [s.size for s in srcs])
    arr = (ctypes.c_void_p * len(srcs))(*[s.ctypes.data for s in srcs])
    check(lib.glx_host_reduce_n(int(op), int(dtype), dst.ctypes.data, arr, len(srcs), int(n)),
          "host_reduce_n")
    return dst
