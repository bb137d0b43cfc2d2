"""Probe: can another process open (and read the end of) an IPC-exported
allocation of a given size?  Two processes, no torch:

    python ipc_size_probe.py export <dir> [flags] &  python ipc_size_probe.py import <dir>

flags: hipExtMallocWithFlags flags (3 = uncached, the device engines'
blocks); none = hipMalloc.

The exporter allocates each size, writes a marker in the last 8 bytes and
the handle to <dir>/h<size>; the importer opens it, reads the marker, closes
it and writes <dir>/ok<size>.  Every step prints with its time."""
import ctypes
import os
import sys
import time

SIZES = [1 << 30, (2 << 30) - (2 << 20), 2 << 30, (2 << 30) + (2 << 20), (4 << 30) + (2 << 20)]
if os.environ.get("PROBE_TORCH"):  # torch's bundled HIP runtime (the product's)
    import torch
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
else:
    hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")


class Handle(ctypes.Structure):  # hipIpcMemHandle_t, passed by value to the open
    _fields_ = [("reserved", ctypes.c_char * 64)]


hip.hipIpcGetMemHandle.argtypes = [ctypes.POINTER(Handle), ctypes.c_void_p]
hip.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), Handle, ctypes.c_uint]
T0 = time.time()


def log(*a):
    print("%7.2f" % (time.time() - T0), *a, flush=True)


def wait_file(path, limit=60):
    t = time.time()
    while not os.path.exists(path):
        if time.time() - t > limit:
            log("gave up waiting for", path)
            sys.exit(3)
        time.sleep(0.05)
    time.sleep(0.05)


def main():
    role, d = sys.argv[1], sys.argv[2]
    assert hip.hipSetDevice(0) == 0
    for n in SIZES:
        if role == "export":
            p = ctypes.c_void_p()
            if len(sys.argv) > 3:
                rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(n),
                                               ctypes.c_uint(int(sys.argv[3])))
            else:
                rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n))
            marker = ctypes.c_uint64(0x5EED0000 + (n >> 20))
            rc2 = hip.hipMemcpy(ctypes.c_void_p(p.value + n - 8), ctypes.byref(marker),
                                ctypes.c_size_t(8), 1)
            h = Handle()
            rc3 = hip.hipIpcGetMemHandle(ctypes.byref(h), p)
            log("export %d bytes: malloc %d memcpy %d handle %d" % (n, rc, rc2, rc3))
            with open(os.path.join(d, "h%d.tmp" % n), "wb") as f:
                f.write(bytes(h))
            os.rename(os.path.join(d, "h%d.tmp" % n), os.path.join(d, "h%d" % n))
            wait_file(os.path.join(d, "ok%d" % n))
            hip.hipFree(p)
        else:
            wait_file(os.path.join(d, "h%d" % n))
            with open(os.path.join(d, "h%d" % n), "rb") as f:
                h = Handle.from_buffer_copy(f.read())
            q = ctypes.c_void_p()
            log("import %d bytes: opening" % n)
            rc = hip.hipIpcOpenMemHandle(ctypes.byref(q), h, 1)
            log("import %d bytes: open rc %d at %s; reading the last 8 bytes" % (n, rc, hex(q.value or 0)))
            v = ctypes.c_uint64(0)
            rc2 = hip.hipMemcpy(ctypes.byref(v), ctypes.c_void_p((q.value or 0) + n - 8),
                                ctypes.c_size_t(8), 2)
            log("import %d bytes: read rc %d value %s (want %s)" % (
                n, rc2, hex(v.value), hex(0x5EED0000 + (n >> 20))))
            hip.hipIpcCloseMemHandle(q)
            open(os.path.join(d, "ok%d" % n), "w").close()
    log(role, "done")


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
