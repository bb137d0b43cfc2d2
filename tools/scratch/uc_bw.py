"""Bandwidth of the glx reduce kernel (dst = a + b, fp32) when its operands
live in uncached / fine-grained / ordinary device memory: the memory kinds the
device-driven engines land peers' data in (xgmi_kernels.hip).  One GPU.

    python tools/uc_bw.py [MiB]
"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import torch

    import gloo_amd
    from gloo_amd import _lib

    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    n = (mib << 20) // 4
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                          ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    kinds = {"normal": 0, "finegrained": 1, "uncached": 3}

    def alloc(kind):
        p = ctypes.c_void_p()
        rc = hip.hipExtMallocWithFlags(ctypes.byref(p), n * 4, kinds[kind])
        assert rc == 0, (kind, rc)
        return p.value

    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    lib = _lib.lib
    for da, sa in (("normal", "normal"), ("normal", "uncached"), ("uncached", "normal"),
                   ("uncached", "uncached"), ("normal", "finegrained"),
                   ("finegrained", "normal")):
        dst = alloc(da)
        a = alloc(sa)
        b = alloc(sa)
        for _ in range(3):
            lib.glx_reduce(1, 5, dst, a, b, n, sp)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record(s)
        for _ in range(reps):
            lib.glx_reduce(1, 5, dst, a, b, n, sp)
        e1.record(s)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / reps / 1e3
        print("dst %-11s srcs %-11s %7.1f us  %6.0f GB/s" % (da, sa, t * 1e6,
                                                            3 * n * 4 / t / 1e9), flush=True)
        for p in (dst, a, b):
            hip.hipFree(p)
    del gloo_amd


if __name__ == "__main__":
    main()
