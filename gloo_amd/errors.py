"""gloo's exception types (gloo/common/error.h, gloo/common/logging.h),
raised from the C ABI's status codes."""
from . import _lib


class Exception(RuntimeError):  # noqa: A001 - mirrors gloo::Exception
    """Base of gloo_amd errors (gloo::Exception, gloo/common/error.h:30)."""


class EnforceNotMet(Exception):
    """A GLOO_ENFORCE check failed (gloo/common/logging.h:21-52)."""


class IoException(Exception):
    """Unrecoverable I/O error: timeout or peer loss (gloo/common/error.h:45).
    The caller must rebuild the context (docs/errors.md)."""


class HipError(Exception):
    """A HIP runtime call failed (CUDA_CHECK analog, gloo/cuda_private.h:25-37)."""


def check(rc, what=""):
    if rc == _lib.OK:
        return
    msg = _lib.last_error()
    if what:
        msg = "%s: %s" % (what, msg)
    if rc in (_lib.ERR_TIMEOUT, _lib.ERR_IO):
        raise IoException(msg)
    if rc == _lib.ERR_HIP:
        raise HipError(msg)
    if rc in (_lib.ERR_ENFORCE, _lib.ERR_INVALID):
        raise EnforceNotMet(msg)
    raise Exception(msg)


def check_handle(h, what):
    if not h:
        msg = _lib.last_error() or "failed"
        low = msg.lower()
        if "timed out" in low or "connection closed" in low:
            raise IoException("%s: %s" % (what, msg))
        raise EnforceNotMet("%s: %s" % (what, msg))
    return h
