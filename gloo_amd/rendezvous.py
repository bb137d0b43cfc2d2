"""Rendezvous: stores and the connected Context (gloo/rendezvous/*).

    store = rendezvous.HashStore()              # ranks are threads
    store = rendezvous.FileStore("/tmp/x")      # ranks are processes
    store = rendezvous.TorchStore(dist_store)   # torch.distributed store
    ctx = rendezvous.Context(rank, size, device)
    ctx.connectFullMesh(store)
"""
import ctypes

from . import _lib
from .errors import check, check_handle

lib = _lib.lib


class Store:
    """gloo::rendezvous::Store (gloo/rendezvous/store.h)."""

    def __init__(self, handle):
        self._h = check_handle(handle, type(self).__name__)

    @property
    def handle(self):
        return self._h

    def set(self, key, data):
        data = bytes(data)
        buf = ctypes.create_string_buffer(data, len(data))
        check(lib.glx_store_set(self._h, key.encode(), buf, len(data)), "Store.set")

    def get(self, key, timeout_ms=30000):
        n = ctypes.c_size_t(0)
        cap = 1 << 16
        buf = ctypes.create_string_buffer(cap)
        check(lib.glx_store_get(self._h, key.encode(), buf, cap, ctypes.byref(n),
                                int(timeout_ms)), "Store.get")
        if n.value > cap:
            buf = ctypes.create_string_buffer(n.value)
            check(lib.glx_store_get(self._h, key.encode(), buf, n.value, ctypes.byref(n),
                                    int(timeout_ms)), "Store.get")
        return buf.raw[: n.value]

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.glx_store_destroy(h)
            self._h = None


class HashStore(Store):
    """In-process store (gloo/rendezvous/hash_store.h:20)."""

    def __init__(self):
        super().__init__(lib.glx_hash_store_create())


class FileStore(Store):
    """Directory-backed store (gloo/rendezvous/file_store.h:19)."""

    def __init__(self, path):
        super().__init__(lib.glx_file_store_create(str(path).encode()))


class PrefixStore(Store):
    """Key-prefixing wrapper (gloo/rendezvous/prefix_store.h)."""

    def __init__(self, prefix, base):
        self._base = base
        super().__init__(lib.glx_prefix_store_create(prefix.encode(), base.handle))


class TorchStore(Store):
    """Bridges a torch.distributed Store (e.g. the TCPStore torchrun creates)
    into the native rendezvous via set/get callbacks."""

    def __init__(self, dist_store):
        self._ds = dist_store

        def _set(user, key, data, n):
            try:
                self._ds.set(key.decode(), ctypes.string_at(data, n) if n else b"")
                return 0
            except Exception:  # noqa: BLE001
                return -1

        def _get(user, key, buf, cap):
            k = key.decode()
            try:
                if not self._ds.check([k]):
                    return -1
                v = self._ds.get(k)
            except Exception:  # noqa: BLE001
                return -1
            if buf and cap:
                ctypes.memmove(buf, v, min(cap, len(v)))
            return len(v)

        self._set_cb = _lib.STORE_SET_FN(_set)
        self._get_cb = _lib.STORE_GET_FN(_get)
        super().__init__(lib.glx_callback_store_create(
            ctypes.cast(self._set_cb, ctypes.c_void_p),
            ctypes.cast(self._get_cb, ctypes.c_void_p), None))


class Context:
    """gloo::rendezvous::Context (gloo/rendezvous/context.h:25-35) bound to
    one HIP device, connected over the in-node xGMI transport."""

    def __init__(self, rank, size, device=-1):
        self._h = check_handle(lib.glx_context_create(int(rank), int(size), int(device)),
                               "Context")
        self._store = None

    @property
    def handle(self):
        return self._h

    @property
    def rank(self):
        return lib.glx_context_rank(self._h)

    @property
    def size(self):
        return lib.glx_context_size(self._h)

    @property
    def device(self):
        return lib.glx_context_device(self._h)

    def connectFullMesh(self, store, device=None):  # noqa: N802 - gloo's name
        """gloo/rendezvous/context.cc:43-113."""
        self._store = store  # keep alive: algorithms exchange through it
        check(lib.glx_context_connect_full_mesh(self._h, store.handle),
              "connectFullMesh")

    connect_full_mesh = connectFullMesh

    def setTimeout(self, seconds_or_ms, ms=False):  # noqa: N802
        """gloo::Context::setTimeout; seconds (float) unless ms=True."""
        val = int(seconds_or_ms if ms else round(seconds_or_ms * 1000))
        check(lib.glx_context_set_timeout(self._h, val), "setTimeout")

    @property
    def base(self):
        """gloo::Context::base (gloo/context.h:33): ranks per group of the
        AllreduceBcube algorithms created afterwards (default 2)."""
        return getattr(self, "_base", 2)

    @base.setter
    def base(self, value):
        check(lib.glx_context_set_base(self._h, int(value)), "base")
        self._base = int(value)

    def getTimeout(self):  # noqa: N802
        """Timeout in seconds."""
        return lib.glx_context_get_timeout(self._h) / 1000.0

    def nextSlot(self, numToSkip=1):  # noqa: N802,N803
        return lib.glx_context_next_slot(self._h, int(numToSkip))

    def ipc_stats(self):
        """IPC imports made and canary-checked, and how many the runtime
        mapped at the base of the exporter's allocation (corrected)."""
        import ctypes
        a, b = ctypes.c_int64(0), ctypes.c_int64(0)
        check(lib.glx_context_ipc_stats(self._h, ctypes.byref(a), ctypes.byref(b)), "ipc_stats")
        return {"imports": a.value, "base_fixups": b.value}

    def peer_info(self, peer):
        """What this rank read at connect about `peer`'s GPU: its device
        ordinal here, whether it is our own GPU, hipDeviceCanAccessPeer and
        the link's hipDevP2PAttrNativeAtomicSupported (None: same GPU or not
        asked), and whether our kernels write peers' flags with stores."""
        import ctypes
        v = (ctypes.c_int * 5)()
        check(lib.glx_context_peer_info(self._h, int(peer), v), "peer_info")
        opt = (lambda x: None if x < 0 else bool(x))
        return {"device": v[0], "same_gpu": bool(v[1]), "can_access_peer": opt(v[2]),
                "native_atomics": opt(v[3]), "flag_stores": bool(v[4])}

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            lib.glx_context_destroy(h)
            self._h = None

    def __del__(self):
        self.close()


class LinkProbe:
    """Measured link ceilings between the context's ranks (glx.h
    glx_link_probe_*): a receive block per rank through the context's own
    canary-checked IPC path.  Creating one is collective.  run() is per rank
    and does not synchronise: barrier before it and take the max time over
    ranks; barrier again before close()."""

    RING, MESH = 0, 1
    DMA, KERNEL = 0, 1

    def __init__(self, ctx, nbytes):
        self._ctx = ctx  # keep alive
        self._h = check_handle(lib.glx_link_probe_create(ctx.handle, int(nbytes)), "LinkProbe")

    def run(self, pattern, engine, blocks=256, reps=5):
        """(seconds on this rank, bytes per round on its busiest link)."""
        import ctypes
        secs, lb = ctypes.c_double(0.0), ctypes.c_size_t(0)
        check(lib.glx_link_probe_run(self._h, int(pattern), int(engine), int(blocks), int(reps),
                                     ctypes.byref(secs), ctypes.byref(lb)), "LinkProbe.run")
        return secs.value, lb.value

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            lib.glx_link_probe_destroy(h)
            self._h = None

    def __del__(self):
        self.close()
