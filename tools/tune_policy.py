"""Cache policy of the reduce kernel's streams, through the product
(glx_tune_reduce's policy code: 0 plain, 1 nt loads+stores, 2 nt loads +
write-through stores, 3 nt loads + plain stores) on the cfg2 workload
(a = a + b and c = a + b, fp32, uniform [-1, 1) inputs) at 16 MiB, 256 MiB and
1 GiB per buffer; prints us per launch (median of timed groups) and
algorithmic TB/s, and checks every policy's result bit for bit against torch.

    python tools/tune_policy.py [MiB ...]   (GPU box)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gloo_amd  # noqa: E402
from gloo_amd import _lib  # noqa: E402

NAMES = {0: "plain", 1: "nt", 2: "nt_ld+wt_st", 3: "nt_ld+plain_st"}


def main():
    out = []
    sizes = [int(x) for x in sys.argv[1:]] or [16, 256, 1024]
    for mib in sizes:
        n = (mib << 20) // 4
        g = torch.Generator(device="cuda").manual_seed(mib)
        a0 = torch.rand(n, device="cuda", generator=g) * 2 - 1
        b = torch.rand(n, device="cuda", generator=g) * 2 - 1
        c = torch.empty_like(a0)
        a = a0.clone()
        ref = a0 + b
        reps = max(8, (4 << 30) // (mib << 20) * 3)
        for inplace in (True, False):
            for pol in (1, 2, 1, 2):
                _lib.lib.glx_tune_reduce(4, 64, pol)
                dst = a if inplace else c
                a.copy_(a0)
                gloo_amd.math.sum(dst, a, b)
                torch.cuda.synchronize()
                ok = bool(torch.equal(dst, ref))
                meds = []
                for _ in range(5):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(reps):
                        gloo_amd.math.sum(dst, a, b)
                    e1.record()
                    torch.cuda.synchronize()
                    meds.append(e0.elapsed_time(e1) / reps * 1e3)
                us = sorted(meds)[len(meds) // 2]
                out.append({"MiB": mib, "inplace": inplace, "policy": NAMES[pol],
                            "us": round(us, 2), "TBps": round(3 * (mib << 20) / us / 1e6, 3),
                            "bit_exact": ok})
                print(json.dumps(out[-1]), flush=True)
    _lib.lib.glx_tune_reduce(4, 64, 4)  # back to auto


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
