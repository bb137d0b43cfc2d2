"""HIP events through the C ABI: the record / query / wait half of the
reference's gloo::CudaStream (gloo/cuda.h:40-120), so a caller can order
its own streams (or the host) after an algorithm that runs on streams
without synchronising the device."""
import ctypes

from . import _lib
from .errors import check


def _stream_handle(stream):
    if stream is None:
        return None
    return ctypes.c_void_p(getattr(stream, "cuda_stream", stream))


class Event:
    def __init__(self):
        h = ctypes.c_void_p()
        check(_lib.lib.glx_event_create(ctypes.byref(h)), "Event")
        self.handle = h

    def record(self, stream=None):
        """Record on `stream` (a torch.cuda.Stream or a raw hipStream_t;
        None = the legacy default stream)."""
        check(_lib.lib.glx_event_record(self.handle, _stream_handle(stream)), "Event.record")

    def query(self):
        """True once everything recorded before it has completed."""
        rc = _lib.lib.glx_event_query(self.handle)
        if rc == _lib.NOT_READY:
            return False
        check(rc, "Event.query")
        return True

    def wait(self, stream=None):
        """Make `stream` wait for this event on the device; with None block
        the calling thread until it completes."""
        check(_lib.lib.glx_event_wait(self.handle, _stream_handle(stream)), "Event.wait")

    def close(self):
        h = getattr(self, "handle", None)
        if h:
            _lib.lib.glx_event_destroy(h)
            self.handle = None

    def __del__(self):
        self.close()
