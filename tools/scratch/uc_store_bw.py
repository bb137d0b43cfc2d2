"""Copy-kernel bandwidth into / out of the memory kinds the engines use, one
process, one GPU: plain hipMalloc, fine-grained and uncached
(hipExtMallocWithFlags).  Tells whether the device engines' slowness on the
shared-GPU rehearsal comes from stores into uncached landing slots.

    python tools/scratch/uc_store_bw.py   (GPU box)
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import gloo_amd  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                      ctypes.c_uint]
KINDS = {"plain": 0x0, "finegrained": 0x1, "uncached": 0x3}
N = 256 << 20


def alloc(flags):
    p = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), N, flags)
    assert rc == 0, rc
    return p.value


def timed(fn, reps=20):
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


def main():
    torch.cuda.init()
    src = torch.empty(N, dtype=torch.uint8, device="cuda").fill_(7)
    bufs = {k: alloc(f) for k, f in KINDS.items()}
    s = torch.cuda.current_stream()
    out = {}
    for blocks in (256, 512, 1024):
        for k, p in bufs.items():
            t = timed(lambda: gloo_amd.kernel_copy(p, src.data_ptr(), N, blocks, s))
            out["store_into_%s_%dwg" % (k, blocks)] = round(N / t / 1e9, 1)
            t = timed(lambda: gloo_amd.kernel_copy(src.data_ptr(), p, N, blocks, s))
            out["load_from_%s_%dwg" % (k, blocks)] = round(N / t / 1e9, 1)
        t = timed(lambda: gloo_amd.peer_copy(bufs["uncached"], 0, src.data_ptr(), 0, N, s))
        out["dma_into_uncached"] = round(N / t / 1e9, 1)
    print(json.dumps(out, indent=1))
    # never hipFree uncached memory: the process exit reclaims it


if __name__ == "__main__":
    main()
