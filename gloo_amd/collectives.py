"""Function-style collective: gloo::allreduce(AllreduceOptions) on device
buffers (gloo/allreduce.h:89-193, gloo/allreduce.cc:97-146).

    opts = AllreduceOptions(context)
    opts.setOutput(t)                  # in place; or setInputs([...]) + setOutputs([...])
    opts.setReduceFunction(ReductionFunction.sum)
    opts.setAlgorithm(AllreduceOptions.Algorithm.RING)
    allreduce(opts)

On device buffers the reduce function is one of the gloo/math.h ops
(ReductionFunction / ReductionType / gloo_amd.math.sum ...): a device cannot
run a host callable.  On host buffers (numpy arrays, CPU tensors, raw host
pointers) any callable works as the reference's AllreduceOptions::Func
(gloo/allreduce.h:36,69,171): fn(c, a, b, n) with raw addresses, c = f(a, b)
over n elements, called in the reference's order on the host
(glx_allreduce_host_fn).  Results are bit-identical to the reference's for
the same inputs, ring and bcube.
"""
import ctypes
import datetime

from . import _lib
from . import math as _math
from .algorithms import ReductionFunction, _as_ptrs, _stream_ptr
from .errors import EnforceNotMet, check

lib = _lib.lib

_MATH_FUNCS = {_math.sum: 1, _math.product: 2, _math.max: 3, _math.min: 4}


class AllreduceOptions:
    """gloo::AllreduceOptions (gloo/allreduce.h:89-193)."""

    class Algorithm:  # gloo/allreduce.h:38-42 (+ RING's result over all links / in one round)
        UNSPECIFIED = 0  # RING's result, data movement chosen by size
        RING = 1
        BCUBE = 2
        RING_MESH = 3
        RING_REPLICATED = 4

    def __init__(self, context):
        self.context = context
        self.algorithm = self.Algorithm.UNSPECIFIED
        self._inputs, self._outputs = [], []
        self.elements = None
        self.dtype = None
        self.op = None
        self.tag = 0
        self.max_segment_size = 0  # 0: the reference's 1 MiB default (allreduce.h:80)
        self.timeout_ms = 0        # 0: the context's timeout
        self.stream = None
        self._in_ptrs = self._out_ptrs = None  # (ctypes array, count), from the setters
        self._any_cuda = False
        self.custom = None  # a host callable fn(c, a, b, n) (setReduceFunction)

    def setAlgorithm(self, algorithm):
        self.algorithm = int(algorithm)

    def setInput(self, buf, elements=None):
        self.setInputs([buf], elements)

    def setInputs(self, bufs, elements=None, dtype=None):
        self._inputs = list(bufs)
        self._in_ptrs = self._sizes(self._inputs, elements, dtype) if self._inputs else None

    def setOutput(self, buf, elements=None):
        self.setOutputs([buf], elements)

    def setOutputs(self, bufs, elements=None, dtype=None):
        self._outputs = list(bufs)
        self._out_ptrs = self._sizes(self._outputs, elements, dtype) if self._outputs else None

    # Assigning the lists goes through the setters, so the pointers allreduce()
    # uses always belong to the buffers the options hold; reading
    # them gives a tuple, so an in-place edit raises instead of being lost
    # (ADVICE r5).
    @property
    def inputs(self):
        return tuple(self._inputs)

    @inputs.setter
    def inputs(self, bufs):
        self.setInputs(bufs)

    @property
    def outputs(self):
        return tuple(self._outputs)

    @outputs.setter
    def outputs(self, bufs):
        self.setOutputs(bufs)

    def _sizes(self, bufs, elements, dtype):
        """Checks the buffers and returns their pointers, taken now as the
        reference's setInput/setOutput take them (gloo/allreduce.h:103-141):
        allreduce() reuses them call after call."""
        ptrs, dt, numel = _as_ptrs(bufs, dtype if dtype is not None else self.dtype)
        if self.dtype is not None and dt != self.dtype:
            raise TypeError("inputs and outputs must share one dtype")
        self.dtype = dt
        if elements is None:
            if numel is None:
                raise ValueError("elements is required with raw pointers")
            elements = numel
        if numel is not None and elements > numel:
            raise ValueError("elements %d exceeds buffer size %d" % (elements, numel))
        self.elements = int(elements)
        self._any_cuda = any(getattr(b, "is_cuda", False)
                             for b in list(self._outputs) + list(self._inputs))
        return (ctypes.c_void_p * max(len(ptrs), 1))(*ptrs), len(ptrs)

    def setReduceFunction(self, fn):
        """ReductionFunction.sum/..., a ReductionType value,
        gloo_amd.math.sum/product/max/min -- or, for host buffers, any
        callable fn(c, a, b, n) on raw addresses (the reference's Func)."""
        self.custom = None
        if isinstance(fn, ReductionFunction):
            if fn.type() not in (1, 2, 3, 4):
                raise EnforceNotMet(
                    "a CUSTOM ReductionFunction is a class algorithm's x = f(x, y); "
                    "gloo::allreduce takes the reference's Func: pass a callable "
                    "fn(c, a, b, n)")
            self.op = fn.type()
        elif isinstance(fn, int) and 1 <= fn <= 4:
            self.op = fn
        elif fn in _MATH_FUNCS:
            self.op = _MATH_FUNCS[fn]
        elif callable(fn):
            self.op, self.custom = None, fn
        else:
            raise EnforceNotMet("reduce function must be a gloo/math.h reduction or a "
                                "callable fn(c, a, b, n); got %r" % (fn,))

    def setTag(self, tag):
        self.tag = int(tag) & 0xFFFFFFFF

    def setMaxSegmentSize(self, nbytes):
        self.max_segment_size = int(nbytes)

    def setTimeout(self, timeout):
        """seconds (float) or datetime.timedelta."""
        if isinstance(timeout, datetime.timedelta):
            timeout = timeout.total_seconds()
        self.timeout_ms = max(1, int(round(float(timeout) * 1000)))

    def setStream(self, stream):
        """Order the work on `stream` (torch.cuda.Stream or a hipStream_t)
        instead of returning with the outputs complete."""
        self.stream = stream


def allreduce(opts):
    """gloo::allreduce(opts) (gloo/allreduce.cc:97-146).  Without a stream
    the call is ordered after the work queued on torch's current stream and
    returns with the outputs complete, like the reference's blocking call."""
    if not opts._outputs:
        raise EnforceNotMet("allreduce: at least one output is required")
    if opts.custom is not None:
        return _allreduce_host_fn(opts)
    op = opts.op if opts.op is not None else 1
    iarr, ni = opts._in_ptrs if opts._inputs else ((ctypes.c_void_p * 1)(), 0)
    oarr, no = opts._out_ptrs
    sync = None
    stream = _stream_ptr(opts.stream)
    if stream is None and opts._any_cuda:
        import torch
        cur = torch.cuda.current_stream()
        if cur.cuda_stream:
            sync, stream = cur, cur.cuda_stream  # ordered on it, then waited for
        else:
            cur.synchronize()  # the null stream: let its queued writes land first
    check(lib.glx_allreduce(opts.context.handle, opts.algorithm, opts.dtype, op,
                            iarr, ni, oarr, no, opts.elements or 0,
                            opts.tag, opts.max_segment_size, opts.timeout_ms, stream),
          "allreduce")
    if sync is not None:
        sync.synchronize()


_REDUCE_FN = _lib.REDUCE_FN  # glx.h glx_reduce_fn: (user, c, a, b, n)


def _allreduce_host_fn(opts):
    """A caller's reduction function on host buffers (glx_allreduce_host_fn):
    the reference's step order on the host, fn(c, a, b, n) per reduction."""
    if opts._any_cuda:
        raise EnforceNotMet("allreduce: a host reduction function needs host buffers "
                            "(a device cannot run it); device buffers take gloo::sum/"
                            "product/max/min")
    user_fn = opts.custom
    errors = []

    def tramp(_user, c, a, b, n):
        if errors:
            return 1
        try:
            user_fn(c, a, b, n)
        except BaseException as e:  # noqa: BLE001 - re-raised after the call
            errors.append(e)
            return 1  # the call stops here (glx.h glx_reduce_fn)
        return 0
    cb = _REDUCE_FN(tramp)
    iarr, ni = opts._in_ptrs if opts._inputs else ((ctypes.c_void_p * 1)(), 0)
    oarr, no = opts._out_ptrs
    es = int(lib.glx_dtype_size(opts.dtype))
    algorithm = opts.algorithm
    if algorithm not in (AllreduceOptions.Algorithm.UNSPECIFIED,
                         AllreduceOptions.Algorithm.RING, AllreduceOptions.Algorithm.BCUBE):
        raise EnforceNotMet("allreduce with a host reduction function: RING or BCUBE")
    rc = lib.glx_allreduce_host_fn(opts.context.handle, algorithm, es,
                                   ctypes.cast(cb, ctypes.c_void_p), None, iarr, ni,
                                   oarr, no, opts.elements or 0, opts.tag,
                                   opts.max_segment_size, opts.timeout_ms)
    if errors:
        raise errors[0]
    check(rc, "allreduce")
