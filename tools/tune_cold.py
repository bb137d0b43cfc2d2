"""The reduce kernel's launch shape and cache policy on the HBM-only loop
bench.py times at N = 1 since round 5 (COLD_PAIRS buffer pairs rotated, so
no launch finds its inputs in the 256 MB Infinity Cache): every (policy,
blocks per CU, unroll) through glx_tune_reduce, in place a = a + b over
256 MiB fp32, us per launch (median of 5 timed groups of 40 launches),
result checked bit for bit against torch once per configuration.  The
round-2/3/4 sweeps (tools/tune_policy.py, tune_reduce.py) timed the launch
back to back over one pair, where write-through stores win by keeping lines
in the Infinity Cache; this one asks which shape is best when nothing is
cached.

    python tools/tune_cold.py [MiB] [f32|f16|bf16]   (GPU box)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gloo_amd  # noqa: E402
from gloo_amd import _lib  # noqa: E402

POLICIES = {0: "plain", 1: "nt", 2: "nt_ld+wt_st", 3: "nt_ld+plain_st"}
PAIRS = 4


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dt = sys.argv[2] if len(sys.argv) > 2 else "f32"
    tdt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[dt]
    n = (mib << 20) // torch.tensor([], dtype=tdt).element_size()
    g = torch.Generator(device="cuda").manual_seed(7)
    pairs = [((torch.rand(n, device="cuda", generator=g) * 2 - 1).to(tdt),
              (torch.rand(n, device="cuda", generator=g) * 2 - 1).to(tdt)) for _ in range(PAIRS)]
    a0 = pairs[0][0].clone()
    # the product's own bits once with the shipped defaults (torch rounds the
    # 16-bit types alike for a sum; fp16's assignment quirk never changes a sum
    # of values in (-1, 1) -- checked against the default launch instead)
    pairs[0][0].copy_(a0)
    gloo_amd.math.sum(pairs[0][0], pairs[0][0], pairs[0][1])
    torch.cuda.synchronize()
    ref = pairs[0][0].clone()
    best = None
    for pol in POLICIES:
        for bpc in (8, 16, 32, 64):
            for unroll in (1, 2, 4, 8):
                _lib.lib.glx_tune_reduce(unroll, bpc, pol)
                a, b = pairs[0]
                a.copy_(a0)
                gloo_amd.math.sum(a, a, b)
                torch.cuda.synchronize()
                ok = bool(torch.equal(a, ref))
                for i in range(PAIRS):
                    x, y = pairs[i]
                    gloo_amd.math.sum(x, x, y)
                meds = []
                for _ in range(5):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for i in range(40):
                        x, y = pairs[i % PAIRS]
                        gloo_amd.math.sum(x, x, y)
                    e1.record()
                    torch.cuda.synchronize()
                    meds.append(e0.elapsed_time(e1) / 40 * 1e3)
                us = sorted(meds)[2]
                rec = {"MiB": mib, "dtype": dt, "policy": POLICIES[pol], "blocks_per_cu": bpc,
                       "unroll": unroll, "us": round(us, 2),
                       "TBps": round(3 * (mib << 20) / us / 1e6, 3), "bit_exact": ok}
                print(json.dumps(rec), flush=True)
                if ok and (best is None or us < best["us"]):
                    best = rec
                # keep the values bounded: restart the accumulated operands
                for x, _ in pairs:
                    x.uniform_(-1, 1)
    _lib.lib.glx_tune_reduce(4, 64, 4)  # back to the shipped defaults (auto policy)
    print(json.dumps({"best": best}), flush=True)


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
