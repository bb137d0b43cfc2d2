#!/usr/bin/env python3
"""The fold kernel (glx_reduce_n: several local pointers into one, the
reference's multi-pointer left fold) over 1 GiB per pointer, fp32: one call
vs consecutive calls over 256 MiB segments, k = 2 and 4 sources, HBM-only
(two rotating sets); us per 1 GiB (median of 5 groups).  Asks whether the
reduce kernel's segmentation pays for the fold too.

    python tools/seg_fold.py   (GPU box)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gloo_amd  # noqa: E402
from gloo_amd.algorithms import ReductionType  # noqa: E402


def timed(fn, reps=6):
    meds = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(reps):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        meds.append(e0.elapsed_time(e1) / reps * 1e3)
    return sorted(meds)[2]


def main():
    n = (1 << 30) // 4
    seg = (256 << 20) // 4
    g = torch.Generator(device="cuda").manual_seed(4)
    for k in (2, 4):
        sets = [[torch.rand(n, device="cuda", generator=g) for _ in range(k)] for _ in range(2)]

        def one(i):
            s = sets[i % 2]
            gloo_amd.math.reduce_n(ReductionType.SUM, s[0], s)

        def segs(i):
            s = sets[i % 2]
            for o in range(0, n, seg):
                gloo_amd.math.reduce_n(ReductionType.SUM, s[0][o:o + seg], [x[o:o + seg] for x in s])
        one(0)
        segs(1)
        torch.cuda.synchronize()
        t1, t4 = timed(one), timed(segs)
        byt = (k + 1) * (1 << 30)
        print(json.dumps({"k": k, "one_call_us": round(t1, 1), "segments_256MiB_us": round(t4, 1),
                          "one_TBps": round(byt / t1 / 1e6, 3),
                          "segments_TBps": round(byt / t4 / 1e6, 3)}), flush=True)
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
