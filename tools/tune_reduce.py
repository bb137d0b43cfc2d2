"""Sweep the reduce kernel's unroll depth and grid cap on the cfg2 workload
(c = a + b, 256 MiB fp32) and a 16 MiB chunk; prints achieved HBM GB/s."""
import faulthandler
import json
import sys

faulthandler.enable()  # a crash prints every thread's stack
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import gloo_amd
from gloo_amd import _lib

res = []
for mib in (256, 16):
    n = (mib << 20) // 4
    a = torch.rand(n, device="cuda"); b = torch.rand(n, device="cuda"); c = torch.empty_like(a)
    for unroll, bpc, nt in [(u, b, t) for t in (0, 1) for u in (1, 2, 4)
                            for b in (1, 2, 3, 4, 8, 64)]:
        if True:
            _lib.lib.glx_tune_reduce(unroll, bpc, nt)
            for inplace in (False, True):
                dst = a if inplace else c
                for _ in range(3):
                    gloo_amd.math.sum(dst, a, b)
                torch.cuda.synchronize()
                e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
                reps = 50 if mib == 256 else 400
                e0.record()
                for _ in range(reps):
                    gloo_amd.math.sum(dst, a, b)
                e1.record(); torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / reps / 1e3
                gbs = 3 * (mib << 20) / t / 1e9
                res.append({"mib": mib, "unroll": unroll, "bpc": bpc, "nt": nt, "inplace": inplace,
                            "us": round(t * 1e6, 2), "GBps": round(gbs, 1)})
                print(json.dumps(res[-1]), flush=True)
best = {}
for r in res:
    k = (r["mib"], r["inplace"])
    if k not in best or r["GBps"] > best[k]["GBps"]:
        best[k] = r
print("BEST", json.dumps(list(best.values())))
