#!/usr/bin/env python3
"""One reduce launch over a whole buffer vs consecutive launches over
segments of it: c = a + b in place, fp32, HBM-only (the buffers rotate so no
launch finds its inputs in the Infinity Cache), total sizes 256 MiB and
1 GiB, segment sizes 32 MiB .. the whole buffer; us per whole buffer (median
of 5 groups).  Round 5 found a single 1 GiB launch 6 % slower than four
256 MiB ones.

    python tools/seg_1GiB.py   (GPU box)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gloo_amd  # noqa: E402


def timed(fn, reps=10):
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
    g = torch.Generator(device="cuda").manual_seed(3)
    for total_mib, npairs in ((256, 4), (1024, 2)):
        n = (total_mib << 20) // 4
        pairs = [(torch.rand(n, device="cuda", generator=g),
                  torch.rand(n, device="cuda", generator=g)) for _ in range(npairs)]
        for seg_mib in (32, 64, 128, 256, 512, 1024):
            if seg_mib > total_mib:
                continue
            seg = (seg_mib << 20) // 4

            def run(i, seg=seg):
                a, b = pairs[i % npairs]
                for k in range(0, n, seg):
                    gloo_amd.math.sum(a[k:k + seg], a[k:k + seg], b[k:k + seg])
            run(0)
            run(1)
            torch.cuda.synchronize()
            us = timed(run)
            print(json.dumps({"total_MiB": total_mib, "segment_MiB": seg_mib,
                              "launches": total_mib // seg_mib, "us": round(us, 1),
                              "TBps": round(3 * (total_mib << 20) / us / 1e6, 3)}), flush=True)
        del pairs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
