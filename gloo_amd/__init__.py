"""gloo_amd -- MI355X-native gloo allreduce hot path.

The drop-in surface of liuxiaotiao/gloo for its data-parallel allreduce:
gloo::Context / rendezvous, gloo::Algorithm with AllreduceRingChunked and
AllreduceHalvingDoubling, the function-style gloo::allreduce(AllreduceOptions)
(ring and bcube), ReductionFunction, and the elementwise reductions of
gloo/math.h -- executed on MI355X GPUs (HIP kernels for gfx950, chunks
moved between the GPUs of a node with hipMemcpyPeerAsync over xGMI).
The native library (libgloo_amd.so, C ABI in include/gloo_amd/glx.h) is
required; there is no CPU fallback.
"""
from . import _lib  # noqa: F401  (raises ImportError if the HIP build is missing)
from . import math, rendezvous  # noqa: F401
from .algorithms import (  # noqa: F401
    AllreduceBcube,
    AllreduceHalvingDoubling,
    AllreduceHalvingDoublingPipelined,
    AllreduceLocal,
    AllreduceRing,
    AllreduceRingChunked,
    HipAllreduceBcube,
    HipAllreduceHalvingDoubling,
    HipAllreduceHalvingDoublingPipelined,
    HipAllreduceLocal,
    HipAllreduceRing,
    HipAllreduceRingChunked,
    ReductionFunction,
    ReductionType,
    device_layout,
    plan,
    plan_sync,
)
from .collectives import AllreduceOptions, allreduce  # noqa: F401
from .events import Event  # noqa: F401
from . import errors  # noqa: F401
from .errors import EnforceNotMet, Exception, HipError, IoException  # noqa: F401,A004

__version__ = _lib.lib.glx_version().decode()
LIB_PATH = _lib.LIB_PATH


def set_copy_split(k):
    """Split each peer copy of algorithms created afterwards over k streams
    (k DMA engines per destination link)."""
    errors.check(_lib.lib.glx_set_copy_split(int(k)), "set_copy_split")


def set_pinned_mirror_limit(nbytes):
    """Host-memory endpoints of algorithms created afterwards: a pageable
    buffer larger than `nbytes` (0: no limit, the default) -- or one the
    runtime cannot pin a whole mirror for -- is staged through an 8 MiB
    pinned bounce block piece by piece instead of a pinned mirror of its
    size (glx.h glx_set_pinned_mirror_limit)."""
    errors.check(_lib.lib.glx_set_pinned_mirror_limit(int(nbytes)), "set_pinned_mirror_limit")


def set_copy_engine(engine, blocks=0):
    """Peer copies of algorithms created afterwards: "dma" (hipMemcpyPeerAsync,
    default) or "kernel" (a copy kernel storing over xGMI into the peer's
    receive region, `blocks` workgroups)."""
    code = {"dma": 0, "kernel": 1}[engine]
    errors.check(_lib.lib.glx_set_copy_engine(code, int(blocks)), "set_copy_engine")


def set_mesh_engine(engine):
    """Engine of mesh-schedule algorithms created afterwards when the ranks
    are on distinct devices or processes: "device" (the two-shot kernel, one
    device-driven launch per rank; default) or "steps" (host-issued copies
    and fold kernels).  Same results either way."""
    code = {"steps": 0, "device": 2}[engine]
    errors.check(_lib.lib.glx_set_mesh_engine(code), "set_mesh_engine")


def set_steps_engine(engine):
    """Engine of ring / halving-doubling / bcube / function-style ring
    algorithms created afterwards when the ranks are on distinct devices or
    processes: "auto" (default: the plan kernel; at every size with one rank
    per GPU, up to 32 MiB per rank when ranks share a GPU, host-issued steps
    above), "device" (the plan kernel, one device-driven
    launch per rank), "host" (host-issued steps) or "dma" (the host-issued
    steps' copies and reduce launches with their hand-offs made on the GPU by
    flag kernels; not for rank threads sharing a device, which then get
    "host").  Same results either way."""
    code = {"host": 0, "device": 3, "dma": 4, "auto": -1}[engine]
    errors.check(_lib.lib.glx_set_steps_engine(code), "set_steps_engine")


def set_engine_streams(policy):
    """Loads and stores of the plan kernel for algorithms created afterwards:
    "auto" (default: "plain", except "fast" for the ring's programs under the
    system-scope flag sync), "plain", or "fast" (nontemporal loads,
    write-through stores).  The one-shot and two-shot kernels
    are always plain."""
    code = {"plain": 0, "fast": 1, "auto": -1}[policy]
    errors.check(_lib.lib.glx_set_engine_streams(code), "set_engine_streams")


def set_max_message_bytes(nbytes):
    """Messages above nbytes go as consecutive pieces, each landing in a
    receive region of its own (glx.h glx_set_max_message_bytes; default
    512 MiB, 0 restores it).  For algorithms created afterwards; every rank
    must use the same value.  Results are unchanged."""
    errors.check(_lib.lib.glx_set_max_message_bytes(int(nbytes)), "set_max_message_bytes")


def max_message_bytes():
    return int(_lib.lib.glx_max_message_bytes())


def set_pipeline_bytes(nbytes):
    """Pipelining below chunk granularity for the host-issued and DMA steps
    engines (glx.h glx_set_pipeline_bytes): messages as pieces of about
    nbytes, each reduced and forwarded on its own; 0 = off.  For algorithms
    created afterwards; every rank must use the same value."""
    errors.check(_lib.lib.glx_set_pipeline_bytes(int(nbytes)), "set_pipeline_bytes")


def pipeline_bytes():
    return int(_lib.lib.glx_pipeline_bytes())


def set_device_sync(mode):
    """Release / acquire around the device engines' flags for algorithms
    created afterwards: "auto" (default: narrow), "system" (L2 written back before
    and invalidated after every flag) or "narrow" (stores completed before a
    flag, the CU's L1 invalidated after a wait: enough because every flag
    publishes data in the receiver's uncached landing slots).

    TEST ONLY: "unsafe_noacquire", "unsafe_norelease", "unsafe_test" and
    "unsafe_cached" are
    deliberately broken positive controls for the suite's stale-data checks
    (glx.h glx_set_device_sync); their results may be wrong."""
    code = _SYNC_MODES[mode]
    errors.check(_lib.lib.glx_set_device_sync(code), "set_device_sync")


_SYNC_MODES = {"auto": -1, "system": 0, "narrow": 1, "unsafe_noacquire": 2,
               "unsafe_norelease": 3, "unsafe_test": 4, "unsafe_cached": 5}
_DEVICE_ENGINE_MODES = {"auto": -1, "off": 0, "on": 1, "shared": 2}


def set_device_engines(mode):
    """Device-driven engines (plan, one-shot and two-shot kernels) for
    algorithms created afterwards (initially GLOO_AMD_DEVICE_ENGINES):
    "auto" (default): only when every rank has a GPU of its own -- ranks
    sharing a GPU run host-issued steps, since their device engines hold the
    GPU's CUs while waiting for each other and can starve other work queued
    ahead of one rank's collective; "shared": also
    processes sharing a GPU while ranks-on-the-GPU x (queues + 1) <= 20,
    where queues is the largest GPU_MAX_HW_QUEUES any rank's process
    published at connect (default 4), for callers that queue no other GPU
    work ahead of a collective there (rehearsals); "on" always; "off" never.
    Every rank decides from the same endpoints and must use the same mode."""
    errors.check(_lib.lib.glx_set_device_engines(_DEVICE_ENGINE_MODES[mode]),
                 "set_device_engines")


def get_device_engines():
    """The current device-engine mode ("auto", "off", "on" or "shared")."""
    code = _lib.lib.glx_get_device_engines()
    return {v: k for k, v in _DEVICE_ENGINE_MODES.items()}[code]


def device_engines_rule(mode, ranks, ranks_per_device, threads_share_device=False,
                        max_hw_queues=4):
    """Whether `mode` gives `ranks` ranks (at most `ranks_per_device` on one
    GPU, the largest GPU_MAX_HW_QUEUES `max_hw_queues`) the device engines:
    the rule set_device_engines applies (glx_device_engines_rule; no GPU)."""
    r = _lib.lib.glx_device_engines_rule(_DEVICE_ENGINE_MODES[mode], int(ranks),
                                         int(ranks_per_device), int(bool(threads_share_device)),
                                         int(max_hw_queues))
    if r < 0:
        errors.check(_lib.ERR_INVALID, "device_engines_rule")
    return bool(r)


def peer_copy(dst_ptr, dst_dev, src_ptr, src_dev, nbytes, stream):
    """nbytes from src (on src_dev) to dst (on dst_dev; may be a peer's
    IPC-mapped memory) by hipMemcpyPeerAsync (the DMA engines), on `stream`
    (torch.cuda.Stream or raw hipStream_t).  Raw pointers: the link probe of
    bench.py and callers holding foreign buffers."""
    from .algorithms import _stream_ptr
    errors.check(_lib.lib.glx_peer_copy(int(dst_ptr), int(dst_dev), int(src_ptr), int(src_dev),
                                        int(nbytes), _stream_ptr(stream)), "peer_copy")


def kernel_copy(dst_ptr, src_ptr, nbytes, blocks, stream):
    """The same copy by the kernel transport's copy kernel: `blocks`
    workgroups of this GPU storing 16-byte vectors into dst."""
    from .algorithms import _stream_ptr
    errors.check(_lib.lib.glx_copy(int(dst_ptr), int(src_ptr), int(nbytes), int(blocks),
                                   _stream_ptr(stream)), "kernel_copy")


def device_count():
    import ctypes
    n = ctypes.c_int(0)
    _lib.lib.glx_device_count(ctypes.byref(n))
    return n.value
