"""Class-style allreduce algorithms on device buffers (gloo/algorithm.h).

    alg = AllreduceRingChunked(context, [t0], count, ReductionFunction.sum)
    alg.run()

Buffers are torch tensors on the context's device (or raw device pointers
with an explicit dtype).  Constructor shape follows
CudaAllreduceRingChunked<T>(context, ptrs, count, streams)
(gloo/cuda_allreduce_ring_chunked.h:22-26).
"""
import ctypes

from . import _lib
from .errors import check, check_handle

lib = _lib.lib

# dtype codes (glx_dtype)
INT8, UINT8, INT32, INT64, UINT64, FLOAT32, FLOAT64, FLOAT16, BFLOAT16 = range(9)


class ReductionType:
    """gloo::ReductionType (gloo/algorithm.h:49-57)."""
    SUM = 1
    PRODUCT = 2
    MAX = 3
    MIN = 4
    CUSTOM = 1000


class ReductionFunction:
    """gloo::ReductionFunction<T> (gloo/algorithm.h:59-96).  The singletons
    sum / product / max / min serve every element type (it comes from the
    buffers).  ReductionFunction(ReductionType.CUSTOM, fn) wraps a caller's
    fn(x, y, n) -- addresses of x and y, n elements, x = f(x, y) in place,
    the reference's Function(T* x, const T* y, size_t n) -- which runs on the
    host: such an algorithm needs host buffers (glx_allreduce_create_host_fn)."""

    def __init__(self, type_, fn=None):
        if type_ == ReductionType.CUSTOM:
            if not callable(fn):
                raise TypeError("a CUSTOM ReductionFunction needs a callable fn(x, y, n)")
        elif fn is not None:
            raise TypeError("only a CUSTOM ReductionFunction takes a function")
        self._type = type_
        self.fn = fn

    def type(self):
        return self._type

    def call(self, x, y, n):
        """x = f(x, y) over n elements at addresses x, y (CUSTOM only)."""
        self.fn(x, y, n)

    def __repr__(self):
        names = {1: "sum", 2: "product", 3: "max", 4: "min", 1000: "custom"}
        return "ReductionFunction.%s" % names[self._type]


ReductionFunction.sum = ReductionFunction(ReductionType.SUM)
ReductionFunction.product = ReductionFunction(ReductionType.PRODUCT)
ReductionFunction.max = ReductionFunction(ReductionType.MAX)
ReductionFunction.min = ReductionFunction(ReductionType.MIN)


def torch_dtype_code(t):
    import torch
    table = {
        torch.int8: INT8, torch.uint8: UINT8, torch.int32: INT32,
        torch.int64: INT64, torch.float32: FLOAT32, torch.float64: FLOAT64,
        torch.float16: FLOAT16, torch.bfloat16: BFLOAT16,
    }
    if hasattr(torch, "uint64"):
        table[torch.uint64] = UINT64
    if t.dtype not in table:
        raise TypeError("unsupported dtype %s" % t.dtype)
    return table[t.dtype]


INT_MAX = (1 << 31) - 1  # the class algorithms' count is a C int

NUMPY_CODES = {"int8": INT8, "uint8": UINT8, "int32": INT32, "int64": INT64,
               "uint64": UINT64, "float32": FLOAT32, "float64": FLOAT64, "float16": FLOAT16}


def _as_ptrs(bufs, dtype, allow_host=True):
    """Buffers -> (list of pointers, dtype code, min numel).  A buffer is a
    device tensor, a host tensor or numpy array (host-memory endpoints:
    staged by the algorithm), or a raw pointer int with an explicit dtype."""
    ptrs, numel = [], None
    for b in bufs:
        if isinstance(b, int):
            if dtype is None:
                raise TypeError("raw pointers need an explicit dtype")
            ptrs.append(b)
            continue
        if hasattr(b, "__array_interface__") and not hasattr(b, "is_cuda"):  # numpy
            if not allow_host:
                raise ValueError("device buffers required")
            if not b.flags["C_CONTIGUOUS"] or not b.flags["WRITEABLE"]:
                raise ValueError("host buffers must be contiguous and writeable")
            code = NUMPY_CODES.get(b.dtype.name)
            if dtype is not None and lib.glx_dtype_size(dtype) == b.itemsize:
                pass  # an explicit dtype reinterprets same-size elements (float16 as uint16 bits)
            elif code is None:
                raise TypeError("unsupported dtype %s" % b.dtype)
            elif dtype is None:
                dtype = code
            elif dtype != code:
                raise TypeError("all buffers must share one dtype")
            ptrs.append(b.ctypes.data)
            numel = b.size if numel is None else min(numel, b.size)
            continue
        if not b.is_cuda and not allow_host:
            raise ValueError("buffers must be device tensors (got %s)" % b.device)
        if not b.is_contiguous():
            raise ValueError("buffers must be contiguous")
        code = torch_dtype_code(b)
        if dtype is None:
            dtype = code
        elif dtype != code and lib.glx_dtype_size(dtype) != b.element_size():
            # an explicit dtype may reinterpret a tensor of the same element
            # size (e.g. uint64 data held in an int64 tensor)
            raise TypeError("all buffers must share one dtype")
        ptrs.append(b.data_ptr())
        numel = b.numel() if numel is None else min(numel, b.numel())
    return ptrs, dtype, numel


def _stream_ptr(s):
    if s is None:
        return None
    if isinstance(s, int):
        return s
    return s.cuda_stream  # torch.cuda.Stream


ALGO_CODES = {"ring_chunked": 0, "halving_doubling": 1, "ring_chunked_mesh": 2,
              # schedules of gloo_amd.allreduce (plan introspection)
              "fn_ring": 3, "fn_ring_mesh": 4, "fn_bcube": 5,
              # one-round variants for small buffers
              "ring_chunked_repl": 6, "fn_ring_repl": 7,
              # creation-time choice among the ring_chunked schedules
              "ring_chunked_auto": 8,
              # class AllreduceRing (whole buffers, each rank's own left fold)
              "ring": 9,
              # class AllreduceBcube (groups of the context's base ranks)
              "bcube": 10,
              # class AllreduceLocal (this rank's pointers only)
              "local": 11}


class Algorithm:
    """gloo::Algorithm (gloo/algorithm.h:20-38)."""

    _algo = None

    def _create(self, *args):
        return lib.glx_allreduce_create(args[0], self._algo, *args[1:])

    def __init__(self, context, ptrs, count=None, fn=None, streams=None, dtype=None):
        if fn is None:
            fn = ReductionFunction.sum
        if not isinstance(ptrs, (list, tuple)):
            ptrs = [ptrs]
        self.context = context
        self._keep = list(ptrs)  # keep tensors alive for the object's lifetime
        pp, dt, numel = _as_ptrs(ptrs, dtype)
        if count is None:
            if numel is None:
                raise ValueError("count is required with raw pointers")
            count = numel
        if numel is not None and count > numel:
            raise ValueError("count %d exceeds buffer size %d" % (count, numel))
        if not 0 <= count <= INT_MAX:
            # the reference's constructors take `const int count`
            # (gloo/allreduce_ring_chunked.h:25, allreduce_halving_doubling.h:
            # 70); ctypes would wrap a larger value silently (2^32 + 5 -> 5)
            raise ValueError(
                "count %d is outside [0, %d], the class algorithms' int count; pass "
                "count= explicitly or use gloo_amd.allreduce (size_t elements)"
                % (count, INT_MAX))
        self.count = int(count)
        self.dtype = dt
        self.fn = fn
        arr = (ctypes.c_void_p * len(pp))(*pp)
        self._hostfn = None
        if fn.type() == ReductionType.CUSTOM:
            self._create_custom(context, arr, len(pp), dt, fn, streams)
            return
        if streams:
            sp = [_stream_ptr(s) for s in streams]
            sarr = (ctypes.c_void_p * len(sp))(*sp)
            ns = len(sp)
        else:
            sarr, ns = None, 0
        self._streams = streams
        self._h = check_handle(
            self._create(context.handle, arr, len(pp), self.count, dt, fn.type(), sarr, ns),
            type(self).__name__)

    def _create_custom(self, context, arr, nptrs, dt, fn, streams):
        """A CUSTOM function: the algorithm's program runs on the host over
        host buffers (glx_allreduce_create_host_fn), calling fn.call(x, y, n)
        where the reference calls fn_->call (x is also the output)."""
        if streams:
            raise ValueError("a CUSTOM reduction function runs on the host: no streams")
        errors = []

        def trampoline(user, c, a, b, n):
            if errors:
                return 1
            try:
                fn.call(c, b, n)  # c == a: x = f(x, y)
            except BaseException as e:  # noqa: BLE001 - re-raised by run()
                errors.append(e)
                return 1  # the run stops here (glx.h glx_reduce_fn)
            return 0
        self._hostfn = (_lib.REDUCE_FN(trampoline), errors)
        self._h = check_handle(
            lib.glx_allreduce_create_host_fn(
                context.handle, self._algo, arr, nptrs, self.count, lib.glx_dtype_size(dt),
                ctypes.cast(self._hostfn[0], ctypes.c_void_p), None),
            type(self).__name__)

    def run(self):
        rc = lib.glx_algorithm_run(self._h)
        if self._hostfn is not None and self._hostfn[1]:
            e = self._hostfn[1][0]
            del self._hostfn[1][:]
            raise e
        check(rc, type(self).__name__ + ".run")

    def run_fed(self):
        """run() on a host buffer that is still being filled (by a transport
        thread calling feed()): each H2D piece goes as soon as it is fed,
        each step waits only for its own range (gloo/transport/tcp/pair.cc:
        385-451 receives into the buffer; here the schedule starts on the
        first bytes).  Blocks until the result is back in host memory."""
        check(lib.glx_algorithm_run_fed(self._h), type(self).__name__ + ".run_fed")

    def feed(self, off, n):
        """Elements [off, off+n) of the host buffer hold their data now (any
        thread; before run_fed() they count for the next run)."""
        check(lib.glx_algorithm_feed(self._h, int(off), int(n)), "feed")

    def done_ranges(self):
        """[(off, n)] element ranges whose results are already in host memory,
        in completion order."""
        cap = 0
        while True:  # ranges keep completing while a run is in flight
            buf = (ctypes.c_int64 * max(2 * cap, 2))()
            k = lib.glx_algorithm_done_ranges(self._h, buf, cap)
            if k < 0:
                check(_lib.ERR_INVALID, "done_ranges")
            if k <= cap:
                return [(buf[2 * i], buf[2 * i + 1]) for i in range(k)]
            cap = 2 * k

    def bytes_sent(self):
        """Bytes this rank moves over peer links per run()."""
        return lib.glx_algorithm_bytes_sent(self._h)

    def engine(self):
        """"steps" (host-issued schedule steps), "oneshot" (the replicated
        schedule as one device-driven kernel per rank), "twoshot" (the mesh
        schedule as one device-driven kernel per rank), "devsteps" (any
        other schedule's step program walked by one device-driven kernel per
        rank), "dmasteps" (the host-issued steps' copies and reduce launches,
        their hand-offs made on the GPU by flag kernels)."""
        return {0: "steps", 1: "oneshot", 2: "twoshot", 3: "devsteps",
                4: "dmasteps", 5: "hostfn"}[lib.glx_algorithm_engine(self._h)]

    def fast_streams(self):
        """True when the plan kernel runs nontemporal loads and write-through
        stores (set_engine_streams; automatic for the ring's programs)."""
        return bool(lib.glx_algorithm_fast_streams(self._h))

    def sync_mode(self):
        """Release / acquire of its device engine around flags: "narrow",
        "system", a test-only "unsafe_*" mode, or None for host-issued steps
        (set_device_sync)."""
        return {1: "narrow", 0: "system", 2: "unsafe_noacquire", 3: "unsafe_norelease",
                4: "unsafe_test", 5: "unsafe_cached", -1: None}[lib.glx_algorithm_sync(self._h)]

    def transport_stats(self):
        """How this algorithm's messages moved since it was created:
        peer_copies (hipMemcpyPeerAsync over xGMI), device_copies
        (hipMemcpyAsync: same-device peers, or after hipMemcpyPeerAsync
        refused a mapping), kernel_copies (copy kernel into the peer's
        memory), device_kernels (device-driven engine launches), bytes, and
        host_folds (multi-pointer host buffers below kOnDeviceThreshold folded
        on the host), done_events (event records after a run's work: none
        for run() on a device engine), flag_kernels (the dmasteps engine's
        hand-off launches)."""
        out = (ctypes.c_int64 * 8)()
        if lib.glx_algorithm_transport_stats(self._h, out, 8) != 8:
            check(_lib.ERR_INVALID, "transport_stats")
        return dict(zip(("peer_copies", "device_copies", "kernel_copies", "device_kernels",
                         "bytes", "host_folds", "done_events", "flag_kernels"), list(out)))

    def record(self, event):
        """Record `event` (gloo_amd.Event) at the end of the last run()'s
        work (on streams[0] when the algorithm has streams)."""
        check(lib.glx_algorithm_record(self._h, event.handle), "record")

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            lib.glx_algorithm_destroy(h)
            self._h = None

    def __del__(self):
        self.close()


class AllreduceRingChunked(Algorithm):
    """gloo::AllreduceRingChunked<T> (gloo/allreduce_ring_chunked.h:19) on
    MI355X: xGMI peer copies + HIP reduce kernel, same chunking and order.

    schedule="auto" (default) picks the data movement by size: replicated
    up to 16 MiB per rank at P=2, 2 MiB at P<=4, 1 MiB at P<=8 when the
    device-driven engines are available (256 KiB otherwise), mesh above,
    the ring from 2 GiB - 64 MiB per rank (the mesh's landing block would
    reach the 2 GiB a peer process can import); the other schedules force
    one.
    schedule="ring" moves chunks around the ring exactly as the
    reference does (one link per direction); schedule="mesh" computes the
    identical result (same chunks, same reduction chain and operand order)
    with every rank exchanging directly with every peer over all links;
    schedule="replicated" (small buffers) computes it in one round: every
    rank receives every peer's buffer and evaluates all chains itself."""

    SCHEDULES = {"ring": "ring_chunked", "mesh": "ring_chunked_mesh",
                 "replicated": "ring_chunked_repl", "auto": "ring_chunked_auto"}

    def __init__(self, context, ptrs, count=None, fn=None, streams=None, dtype=None,
                 schedule="auto"):
        if schedule not in self.SCHEDULES:
            raise ValueError("schedule must be one of %s" % sorted(self.SCHEDULES))
        self._algo = ALGO_CODES[self.SCHEDULES[schedule]]
        self.schedule = schedule
        super().__init__(context, ptrs, count, fn, streams, dtype)


class AllreduceHalvingDoubling(Algorithm):
    """gloo::AllreduceHalvingDoubling<T> (gloo/allreduce_halving_doubling.h:37)."""
    _algo = ALGO_CODES["halving_doubling"]


class AllreduceRing(Algorithm):
    """gloo::AllreduceRing<T> (gloo/allreduce_ring.h:20): every rank ends
    with its own left fold x[r] op x[r-1] op ... op x[r-P+1] of the ranks'
    (locally reduced) buffers, as the reference's P-1 forwarding rounds
    compute it -- so float results may differ between ranks, exactly as in
    the reference.  The data moves in one round over every link (each rank
    sends its buffer to every peer) instead of P-1 dependent ring rounds."""
    _algo = ALGO_CODES["ring"]


class AllreduceBcube(Algorithm):
    """gloo::AllreduceBcube<T> (gloo/allreduce_bcube.h:256): log_base(P)
    reduce-scatter steps within groups of `context.base` ranks (default 2,
    gloo::Context::base), then the all-gather retracing them -- the
    reference's groups, ranges and reduction order exactly."""
    _algo = ALGO_CODES["bcube"]


class AllreduceLocal(Algorithm):
    """gloo::AllreduceLocal<T> (gloo/allreduce_local.cc:21-31): this rank's
    pointers folded into ptrs[0] (((p0 op p1) op p2) ...) and copied back to
    the others; nothing is exchanged with other ranks."""
    _algo = ALGO_CODES["local"]


class AllreduceHalvingDoublingPipelined(AllreduceHalvingDoubling):
    """gloo::CudaAllreduceHalvingDoublingPipelined<T>
    (gloo/cuda_allreduce_halving_doubling_pipelined.h:13-27): halving-doubling
    with the local broadcast pipelined into the reduce.  Same result bits;
    the device-driven schedule overlaps its steps either way."""
    pipelined = True


# The device classes under the names the reference's GPU path uses.
HipAllreduceRingChunked = AllreduceRingChunked
HipAllreduceHalvingDoubling = AllreduceHalvingDoubling
HipAllreduceHalvingDoublingPipelined = AllreduceHalvingDoublingPipelined
HipAllreduceRing = AllreduceRing
HipAllreduceBcube = AllreduceBcube
HipAllreduceLocal = AllreduceLocal


DEFAULT_MIN_PIECE_BYTES = 4 << 20


def plan(algo, rank, size, count, with_folds=False, esize=4, max_segment_size=0,
         min_piece_bytes=DEFAULT_MIN_PIECE_BYTES):
    """The step program of one rank (host logic, no GPU).  algo: a key of
    ALGO_CODES.  The fn_* schedules also depend on the element size, the
    options' maxSegmentSize (0: default) and the ring's device piece size
    (0: the reference's own segments).  Returns (steps as 8-tuples,
    scratch_elems[, fold sources])."""
    scratch = ctypes.c_int64(0)
    if algo.startswith("bcube"):  # "bcube" or "bcube:<base>"
        base = int(algo.split(":")[1]) if ":" in algo else 2
        n = lib.glx_plan_bcube(rank, size, count, base, None, 0, ctypes.byref(scratch))
        if n < 0:
            check(_lib.ERR_INVALID, "plan")
        buf = (ctypes.c_int64 * (8 * max(n, 1)))()
        lib.glx_plan_bcube(rank, size, count, base, buf, n, ctypes.byref(scratch))
        steps = [tuple(buf[8 * i: 8 * i + 8]) for i in range(n)]
        return (steps, scratch.value, {}) if with_folds else (steps, scratch.value)
    code = ALGO_CODES[algo]
    args = (code, rank, size, count, esize, max_segment_size, min_piece_bytes)
    n = lib.glx_plan_ex(*args, None, 0, ctypes.byref(scratch))
    if n < 0:
        check(_lib.ERR_INVALID, "plan")
    buf = (ctypes.c_int64 * (8 * max(n, 1)))()
    lib.glx_plan_ex(*args, buf, n, ctypes.byref(scratch))
    steps = [tuple(buf[8 * i: 8 * i + 8]) for i in range(n)]
    if not with_folds:
        return steps, scratch.value
    folds = {}
    for st in steps:
        if st[0] == 5:
            k = lib.glx_plan_fold_ex(*args, st[5], None, 0)
            fb = (ctypes.c_int64 * max(k, 1))()
            lib.glx_plan_fold_ex(*args, st[5], fb, k)
            folds[st[5]] = list(fb[:k])
    return steps, scratch.value, folds


def device_layout(algo, rank, size, count, esize=4, max_slices=256):
    """Geometry the device-driven engines (one-shot: replicated schedules,
    two-shot: mesh schedules) derive from the compiled plan (host logic, no
    GPU): dict with G, slice, max_len, jobs [(off, len, chain)] (one-shot),
    ranges [(off, len)] by owner and my_chain (two-shot)."""
    code = ALGO_CODES[algo]
    n = lib.glx_device_layout(code, rank, size, count, esize, max_slices, None, 0)
    if n < 0:
        check(_lib.ERR_INVALID, "device_layout")
    b = (ctypes.c_int64 * n)()
    lib.glx_device_layout(code, rank, size, count, esize, max_slices, b, n)
    v = list(b)
    K = 8
    G, slice_, max_len, njobs = v[:4]
    at = 4
    job_off, job_len = v[at:at + K], v[at + K:at + 2 * K]
    at += 2 * K
    chains = [v[at + q * K: at + q * K + size] for q in range(K)]
    at += K * K
    r_off, r_len = v[at:at + K], v[at + K:at + 2 * K]
    at += 2 * K
    my_chain = v[at:at + size]
    return {"G": G, "slice": slice_, "max_len": max_len,
            "jobs": [(job_off[q], job_len[q], chains[q]) for q in range(njobs)],
            "ranges": [(r_off[c], r_len[c]) for c in range(size)], "my_chain": my_chain}


def plan_sync(algo, rank, size, count, G, esize=4, max_segment_size=0,
              min_piece_bytes=DEFAULT_MIN_PIECE_BYTES):
    """The plan kernel's bookkeeping for one rank with G workgroups
    (glx_plan_sync, host logic): dict with bounds (segment bounds), slice,
    safe, slots (landing slots per channel), steps [(channel, seg0, seg1,
    seq, per_run, fuse, rseq, rper_run, keep, pre, pre0, pre1)] (fuse: the
    SEND a REDUCE/COPY forwards in the same pass, or the step a SEND is done
    in, -1 otherwise; rseq/rper_run: the message a REDUCE/COPY reads; keep: 0
    for a fused REDUCE whose result (a partial one's overlap) only goes to
    the peer; pre/pre0/pre1: partial reduce-and-forward, the overlap's
    segments [pre0, pre1) -- plan.h StepSync)."""
    code = ALGO_CODES[algo]
    args = (code, rank, size, count, esize, max_segment_size, min_piece_bytes, G)
    nb = ctypes.c_int64(0)
    info = (ctypes.c_int64 * 3)()
    n = lib.glx_plan_sync(*args, None, 0, ctypes.byref(nb), info, None, 0)
    if n < 0:
        check(_lib.ERR_INVALID, "plan_sync")
    bb = (ctypes.c_int64 * max(nb.value, 1))()
    sb = (ctypes.c_int64 * max(12 * n, 1))()
    lib.glx_plan_sync(*args, bb, nb.value, ctypes.byref(nb), info, sb, 12 * n)  # int64 slots
    return {"bounds": list(bb[:nb.value]), "slice": info[0], "safe": bool(info[1]),
            "slots": info[2], "steps": [tuple(sb[12 * i:12 * i + 12]) for i in range(n)]}


def stage_plan(algo, rank, size, count, esize=4, max_piece=None):
    """Host-memory staging of a plan (glx_plan_stage): (h2d pieces [(off,
    len)] in issue order, copy-backs [(step, off, len)], step -1 = after the
    last step)."""
    code = ALGO_CODES[algo]
    if max_piece is None:
        max_piece = max(1, (8 << 20) // esize)
    nd = ctypes.c_int64(0)
    n = lib.glx_plan_stage(code, rank, size, count, esize, max_piece, None, 0, None, 0,
                           ctypes.byref(nd))
    if n < 0:
        check(_lib.ERR_INVALID, "stage_plan")
    h = (ctypes.c_int64 * (2 * max(n, 1)))()
    d = (ctypes.c_int64 * (3 * max(nd.value, 1)))()
    lib.glx_plan_stage(code, rank, size, count, esize, max_piece, h, n, d, nd.value,
                       ctypes.byref(nd))
    return ([(h[2 * i], h[2 * i + 1]) for i in range(n)],
            [(d[3 * i], d[3 * i + 1], d[3 * i + 2]) for i in range(nd.value)])
