#!/usr/bin/env python3
"""Launch-shape sweep of the reduce kernel for 16-bit types (fp16 / bf16,
256 MiB in place, as bench.py --dtype f16|bf16 times it): unroll x
workgroups-per-CU cap, via glx_tune_reduce.  fp32's shape (unroll 4, 64
WGs/CU) was tuned in round 1 (tools/tune_reduce.py); 16-bit types do more
VALU work per byte (widen, op, round, the fp16 assignment rule)."""
import json
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import gloo_amd
    from gloo_amd import _lib
    out = {}
    n = (256 << 20) // 2
    for dt in (torch.float16, torch.bfloat16):
        a = (torch.rand(n, device="cuda") * 2 - 1).to(dt)
        b = (torch.rand(n, device="cuda") * 2 - 1).to(dt)
        s = torch.cuda.current_stream()
        for unroll in (2, 4, 8):
            for bpc in (8, 16, 32, 64):
                _lib.lib.glx_tune_reduce(unroll, bpc, 4)
                for _ in range(5):
                    gloo_amd.math.sum(a, a, b, stream=s)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(50):
                    gloo_amd.math.sum(a, a, b, stream=s)
                e1.record(s)
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / 50 * 1e3
                out["%s_u%d_b%d" % (str(dt).split(".")[-1], unroll, bpc)] = round(us, 2)
        _lib.lib.glx_tune_reduce(4, 64, 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
