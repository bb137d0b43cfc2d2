"""Write-through vs the current stores for the fold (reduce_n) and copy
kernels, through the product, uniform random fp32.  Run once per setting of
GLOO_AMD_FOLD_WT / GLOO_AMD_COPY_WT (read when the library loads):

    GLOO_AMD_FOLD_WT=0 GLOO_AMD_COPY_WT=0 python tools/scratch/fold_copy_wt.py
    GLOO_AMD_FOLD_WT=1 GLOO_AMD_COPY_WT=1 python tools/scratch/fold_copy_wt.py
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


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    meds = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        meds.append(e0.elapsed_time(e1) / reps * 1e3)
    return sorted(meds)[2]


def main():
    tag = "fold_wt=%s copy_wt=%s" % (os.environ.get("GLOO_AMD_FOLD_WT", "0"),
                                      os.environ.get("GLOO_AMD_COPY_WT", "0"))
    s = torch.cuda.current_stream()
    for mib in (16, 256):
        n = (mib << 20) // 4
        reps = 200 if mib == 16 else 20
        g = torch.Generator(device="cuda").manual_seed(mib)
        srcs = [torch.rand(n, device="cuda", generator=g) * 2 - 1 for _ in range(8)]
        dst = torch.empty_like(srcs[0])
        for k in (2, 4, 8):
            us = timed(lambda: gloo_amd.math.reduce_n(gloo_amd.ReductionType.SUM, dst, srcs[:k]),
                       reps)
            ref = srcs[0].clone()
            for j in range(1, k):
                ref = ref + srcs[j]
            ok = bool(torch.equal(dst, ref))
            print(json.dumps({"set": tag, "kernel": "reduce_n", "k": k, "MiB": mib,
                              "us": round(us, 2),
                              "TBps": round((k + 1) * (mib << 20) / us / 1e6, 3),
                              "bit_exact": ok}), flush=True)
        p = ctypes.c_void_p()
        assert hip.hipExtMallocWithFlags(ctypes.byref(p), mib << 20, 3) == 0
        for what, dptr in (("plain", dst.data_ptr()), ("uncached", p.value)):
            us = timed(lambda: gloo_amd.kernel_copy(dptr, srcs[0].data_ptr(), mib << 20, 256, s),
                       reps)
            print(json.dumps({"set": tag, "kernel": "copy_256wg", "into": what, "MiB": mib,
                              "us": round(us, 2),
                              "TBps": round(2 * (mib << 20) / us / 1e6, 3)}), flush=True)
        ok = bool(torch.equal(dst, srcs[0]))
        print(json.dumps({"set": tag, "copy_bit_exact": ok}), flush=True)


if __name__ == "__main__":
    main()
