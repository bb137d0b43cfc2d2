"""CPU: the C-ABI library loads, exports every symbol include/gloo_amd/glx.h
declares, and its host logic (stores, rendezvous, errors) works without a
GPU.  No compute calls here."""
import ctypes
import os
import re
import threading

import pytest

import gloo_amd
from gloo_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gloo_amd", "glx.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(glx_[a-z0-9_]+)\s*\(", text)) -
                  {"glx_store_set_fn", "glx_store_get_fn"})


def test_every_declared_symbol_is_exported():
    syms = declared_symbols()
    assert len(syms) >= 25
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    bound = {name for name, _, _ in _lib.SIGNATURES}
    assert set(syms) <= bound, set(syms) - bound


def test_version_and_dtype_sizes():
    assert gloo_amd.__version__ == "0.1.0"
    sizes = [_lib.lib.glx_dtype_size(d) for d in range(9)]
    assert sizes == [1, 1, 4, 8, 8, 4, 8, 2, 2]
    assert _lib.lib.glx_dtype_size(42) == 0


def test_reduce_rejects_bad_arguments_without_gpu():
    with pytest.raises(gloo_amd.EnforceNotMet):
        gloo_amd.errors.check(_lib.lib.glx_reduce(99, 5, None, None, None, 0, None))
    with pytest.raises(gloo_amd.EnforceNotMet):
        gloo_amd.errors.check(_lib.lib.glx_reduce(1, 99, None, None, None, 0, None))
    with pytest.raises(gloo_amd.EnforceNotMet):
        gloo_amd.errors.check(_lib.lib.glx_reduce(1, 5, None, None, None, 10, None))


def test_hash_store_and_prefix_store():
    s = gloo_amd.rendezvous.HashStore()
    s.set("k", b"v" * 70000)
    assert s.get("k") == b"v" * 70000
    p = gloo_amd.rendezvous.PrefixStore("pre", s)
    p.set("a", b"1")
    assert s.get("pre/a") == b"1"
    with pytest.raises(gloo_amd.IoException, match="Timed out"):
        s.get("missing", timeout_ms=20)


def test_file_store(tmp_path):
    s = gloo_amd.rendezvous.FileStore(str(tmp_path / "store"))
    s.set("rank/0", b"\x00\x01payload")
    s2 = gloo_amd.rendezvous.FileStore(str(tmp_path / "store"))
    assert s2.get("rank/0") == b"\x00\x01payload"
    with pytest.raises(gloo_amd.IoException):
        s2.get("nope", timeout_ms=20)


def test_context_validation():
    with pytest.raises(gloo_amd.EnforceNotMet):
        gloo_amd.rendezvous.Context(2, 2)
    c = gloo_amd.rendezvous.Context(0, 1)
    assert (c.rank, c.size) == (0, 1)
    c.setTimeout(1.5)
    assert c.getTimeout() == 1.5
    assert [c.nextSlot(), c.nextSlot(3), c.nextSlot()] == [0, 1, 4]


@pytest.mark.parametrize("P", [2, 5])
def test_connect_full_mesh_threads(P):
    """Endpoint exchange + shared-memory control blocks, ranks as threads
    (gloo/rendezvous/context.cc:43-113); no GPU calls are needed for it."""
    store = gloo_amd.rendezvous.HashStore()
    errs, ctxs = [], [None] * P

    def body(r):
        try:
            c = gloo_amd.rendezvous.Context(r, P)
            c.connectFullMesh(store)
            ctxs[r] = c
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=body, args=(r,)) for r in range(P)]
    [t.start() for t in ts]
    [t.join(30) for t in ts]
    assert not errs, errs
    assert all(c is not None for c in ctxs)
    # control-block names are unlinked once everyone has mapped them
    leftovers = [f for f in os.listdir("/dev/shm") if f.startswith("glx.%d." % os.getpid())]
    assert not leftovers


def test_algorithm_needs_connected_context():
    c = gloo_amd.rendezvous.Context(0, 2)
    with pytest.raises(gloo_amd.EnforceNotMet, match="connect"):
        gloo_amd.AllreduceRingChunked(c, [1 << 20], count=16, dtype=5)


@pytest.mark.parametrize("count", [-1, 1 << 31, (1 << 32) + 5])
def test_class_count_outside_c_int_is_refused(count):
    """The class algorithms take the reference's `const int count`
    (gloo/allreduce_ring_chunked.h:25): a count ctypes would wrap (2^32 + 5
    -> 5, a silent partial reduce) is refused before any native call; the C
    ABI refuses a negative one itself."""
    c = gloo_amd.rendezvous.Context(0, 2)
    for cls in (gloo_amd.AllreduceRingChunked, gloo_amd.AllreduceHalvingDoubling):
        with pytest.raises(ValueError, match="int count"):
            cls(c, [1 << 20], count=count, dtype=0)
    arr = (ctypes.c_void_p * 1)(1 << 20)
    assert not _lib.lib.glx_allreduce_ring_chunked_create(c.handle, arr, 1, -1, 0, 1, None, 0)
    assert "count" in _lib.lib.glx_last_error().decode()


def test_library_never_registers_or_copies_caller_host_pages():
    """DESIGN.md 9 (the round-3 illegal address): the library must not hand
    a caller's host pages to the runtime.  It imports neither
    hipHostRegister nor hipHostUnregister, and every host<->device copy of
    the staging code reads or writes a pointer that is pinned: the caller's
    own when already pinned (isPinnedHost), else a mirror or bounce block the
    library took from hipHostMalloc."""
    import shutil
    import subprocess
    nm = shutil.which("nm")
    if nm is None:
        pytest.skip("no nm")
    out = subprocess.run([nm, "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    imported = {line.split()[-1].split("@")[0] for line in out.splitlines() if line.strip()}
    assert "hipHostMalloc" in imported  # the mirrors' allocator (sanity: nm saw the imports)
    assert not {"hipHostRegister", "hipHostUnregister"} & imported
    # the staging copies: the host side is `.dma` (pinned by construction),
    # a mirror / bounce block (b.p, its D2H half `out`), or a pointer that
    # passed isPinnedHost (src, outDma)
    src = open(os.path.join(ROOT, "gloo_amd", "csrc", "executor_host.cc")).read()
    copies = re.findall(r"hipMemcpyAsync\(([^;]*?)\);", src, flags=re.S)
    assert copies
    for args in copies:
        a = [x.strip() for x in args.split(",")]
        kind = a[3]
        host = a[1] if kind == "hipMemcpyHostToDevice" else a[0]
        if kind not in ("hipMemcpyHostToDevice", "hipMemcpyDeviceToHost"):
            continue
        assert re.search(r"\.dma\b|\bb\.p\b|\bsrc\b|\bout\b|outDma\[i\]", host), (host, args)


# (ranks, ranks per GPU, threads share a GPU, largest GPU_MAX_HW_QUEUES) ->
# device engines under (auto, shared, on, off).  8 x 1 is the configuration
# whose collectives starved a GEMM queued ahead of one rank's collective
# (profiles/r9j_*, r9l_*); 8 x 2 time-slices the queues
# (profiles/r7g_queue_sweep.txt); 4 x 2 fits the queue budget.
ENGINE_RULE = [
    ((8, 8, False, 1), (False, True, True, False)),
    ((8, 8, False, 2), (False, False, True, False)),
    ((4, 4, False, 2), (False, True, True, False)),
    ((4, 4, False, 4), (False, True, True, False)),
    ((8, 8, False, 4), (False, False, True, False)),
    ((4, 2, True, 4), (False, False, True, False)),   # threads of one process
    ((8, 1, False, 4), (True, True, True, False)),    # the node: one rank per GPU
    ((2, 1, False, 1), (True, True, True, False)),
    ((1, 1, False, 4), (False, False, False, False)),  # nothing to exchange
]


@pytest.mark.parametrize("shape,expect", ENGINE_RULE)
def test_device_engine_rule(shape, expect):
    """The chooser every rank applies to the context's endpoints
    (HipPlanExecutor::deviceEnginesRule via glx_device_engines_rule): the
    automatic mode gives the device engines only to ranks with a GPU of
    their own, whatever the queue count; the shared mode also to processes
    sharing a GPU within ranks x (queues + 1) <= 20."""
    ranks, per_dev, threads, queues = shape
    got = tuple(gloo_amd.device_engines_rule(m, ranks, per_dev, threads, queues)
                for m in ("auto", "shared", "on", "off"))
    assert got == expect, (shape, got)


def test_device_engine_mode_round_trip_and_rejects():
    before = gloo_amd.get_device_engines()
    try:
        for m in ("shared", "on", "off", "auto"):
            gloo_amd.set_device_engines(m)
            assert gloo_amd.get_device_engines() == m
    finally:
        gloo_amd.set_device_engines(before)
    with pytest.raises(gloo_amd.EnforceNotMet):
        gloo_amd.errors.check(_lib.lib.glx_set_device_engines(3))
    with pytest.raises(gloo_amd.EnforceNotMet):
        gloo_amd.device_engines_rule("auto", 4, 5)  # more ranks on a GPU than ranks


def test_steps_engine_setter_takes_every_engine_and_rejects_others():
    """glx_set_steps_engine: automatic, host-issued steps, the plan kernel and
    the DMA steps engine (GLX_ENGINE_DMASTEPS); anything else is refused."""
    try:
        for e in ("host", "device", "dma", "auto"):
            gloo_amd.set_steps_engine(e)
        for code in (-1, 0, 3, 4):
            assert _lib.lib.glx_set_steps_engine(code) == 0
        for code in (1, 2, 5, -2):
            with pytest.raises(gloo_amd.EnforceNotMet):
                gloo_amd.errors.check(_lib.lib.glx_set_steps_engine(code))
    finally:
        gloo_amd.set_steps_engine("auto")
    header = open(os.path.join(ROOT, "include", "gloo_amd", "glx.h")).read()
    assert "#define GLX_ENGINE_DMASTEPS 4" in header


def test_device_engine_mode_from_environment():
    """GLOO_AMD_DEVICE_ENGINES sets the initial mode (the rehearsal harness's
    opt-in); unset means automatic."""
    import subprocess
    import sys
    code = "import gloo_amd; print(gloo_amd.get_device_engines())"
    for val, want in (("shared", "shared"), ("off", "off"), (None, "auto")):
        env = dict(os.environ)
        env.pop("GLOO_AMD_DEVICE_ENGINES", None)
        if val is not None:
            env["GLOO_AMD_DEVICE_ENGINES"] = val
        out = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT,
                             capture_output=True, text=True, timeout=60)
        assert out.returncode == 0, out.stderr
        assert out.stdout.strip() == want


def test_allreduce_options_assignment_goes_through_the_setters():
    """allreduce() uses the pointers taken by setInputs /
    setOutputs; assigning opts.inputs / opts.outputs must refresh them, not
    leave the old buffers' pointers behind."""
    import numpy as np
    ctx = object()
    opts = gloo_amd.AllreduceOptions(ctx)
    a, b = np.zeros(8, np.float32), np.ones(16, np.float32)
    opts.setOutputs([a])
    assert opts._out_ptrs[0][0] == a.ctypes.data and opts.elements == 8
    opts.outputs = [b]
    assert opts._out_ptrs[0][0] == b.ctypes.data and opts.elements == 16
    assert opts.outputs == (b,) and opts.outputs is not opts._outputs
    with pytest.raises(AttributeError):
        opts.outputs.append(a)  # an in-place edit raises, never lost
    opts.inputs = [b.copy()]
    assert opts._in_ptrs[1] == 1
    opts.inputs = []
    assert opts._in_ptrs is None and opts.inputs == ()


def test_reduce_tuning_is_atomic_across_threads():
    """the reduce kernel's process-wide settings are written by
    glx_tune_reduce while rank threads launch; every read sees a value some
    thread wrote (std::atomic, reduce_kernels.hip), never a torn or stale
    default, and the defaults come back."""
    u, b, p = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    assert _lib.lib.glx_reduce_tuning(ctypes.byref(u), ctypes.byref(b), ctypes.byref(p)) == 0
    defaults = (u.value, b.value, p.value)
    assert defaults == (4, 64, 4)
    choices = [(1, 8, 0), (2, 16, 1), (4, 32, 2), (8, 48, 3), (4, 64, 4)]
    seen, errs = [], []

    def worker(k):
        uu, bb, pp = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        for i in range(3000):
            c = choices[(k + i) % len(choices)]
            if _lib.lib.glx_tune_reduce(*c) != 0:
                errs.append(c)
            _lib.lib.glx_reduce_tuning(ctypes.byref(uu), ctypes.byref(bb), ctypes.byref(pp))
            seen.append((uu.value, bb.value, pp.value))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    try:
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    finally:
        assert _lib.lib.glx_tune_reduce(*defaults) == 0
    assert not errs
    assert {s[0] for s in seen} <= {c[0] for c in choices}
    assert {s[1] for s in seen} <= {c[1] for c in choices}
    assert {s[2] for s in seen} <= {c[2] for c in choices}
    assert _lib.lib.glx_reduce_tuning(ctypes.byref(u), ctypes.byref(b), ctypes.byref(p)) == 0
    assert (u.value, b.value, p.value) == defaults
    with pytest.raises(gloo_amd.EnforceNotMet):
        gloo_amd.errors.check(_lib.lib.glx_tune_reduce(3, 64, 4))


def test_device_sync_modes_round_trip_and_reject():
    """The product's modes (auto, system, narrow) and the test-only broken
    positive controls (unsafe_*: kernels.h kSyncNoAcquire .. kSyncUnsafe) are
    accepted; anything else is refused."""
    try:
        for m in ("system", "narrow", "unsafe_noacquire", "unsafe_norelease", "unsafe_test",
                  "unsafe_cached", "auto"):
            gloo_amd.set_device_sync(m)
        for code in (6, -2):
            with pytest.raises(gloo_amd.EnforceNotMet):
                gloo_amd.errors.check(_lib.lib.glx_set_device_sync(code))
        with pytest.raises(KeyError):
            gloo_amd.set_device_sync("broken")
    finally:
        gloo_amd.set_device_sync("auto")
