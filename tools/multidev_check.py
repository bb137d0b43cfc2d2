#!/usr/bin/env python3
"""Hardware check of SURVEY 8f #4 -- one rank's pointers on several GPUs --
for boxes with more than one GPU visible (the GPU test boxes have one, so
tests/test_allreduce_gpu.py::test_multi_device_pointers_in_one_rank skips
there).  bench.py runs this as a child process when torch sees >= 2 devices
and puts the result in its JSON line ("multi_device_pointers").

The reference's multi-device CUDA ranks (gloo/cuda_collectives_native.h:24-151:
CudaLocalNativeReduce / CudaLocalNativeBroadcast) fold the local pointers
across devices and broadcast the result back.  Here: 2 thread-ranks, each
with k pointers on devices 0..k-1, ring_chunked and halving_doubling.  The
inputs are small integers in fp32 / int32, so every reduction order gives
the same bits and torch (CPU, int64) is the checker -- no oracle needed.

Prints one JSON line: {"devices": k, "ok": bool, "cases": [...]}.
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# self-test of this script on a one-GPU box: every "device" is device 0
SAME_DEVICE = len(sys.argv) > 1 and sys.argv[1] == "--same-device"
sys.path.insert(0, ROOT)


def run_case(torch, gloo_amd, algo, k, n, dtype, seed):
    P = 2
    g = torch.Generator().manual_seed(seed)
    ins = [[torch.randint(-1000, 1000, (n,), generator=g, dtype=torch.int64) for _ in range(k)]
           for _ in range(P)]
    expect = sum(x for row in ins for x in row)
    dev = (lambda i: 0) if SAME_DEVICE else (lambda i: i)
    bufs = [[ins[r][i].to(dtype).to("cuda:%d" % dev(i)) for i in range(k)] for r in range(P)]
    for d in range(k):
        torch.cuda.synchronize(dev(d))
    store = gloo_amd.rendezvous.HashStore()
    errors = [None] * P

    def rank_fn(r):
        try:
            ctx = gloo_amd.rendezvous.Context(r, P, 0)
            ctx.setTimeout(30)
            ctx.connectFullMesh(store)
            cls = (gloo_amd.AllreduceHalvingDoubling if algo == "halving_doubling"
                   else gloo_amd.AllreduceRingChunked)
            alg = cls(ctx, bufs[r])
            for _ in range(2):  # the second run reuses the algorithm's state
                for i in range(k):
                    bufs[r][i].copy_(ins[r][i].to(dtype))
                    torch.cuda.synchronize(dev(i))
                alg.run()
            alg.close()
        except BaseException as e:  # noqa: BLE001 - reported
            errors[r] = "%s: %s" % (type(e).__name__, str(e)[:200])

    threads = [threading.Thread(target=rank_fn, args=(r,), daemon=True) for r in range(P)]
    t0 = time.time()
    for t in threads:
        t.start()
    for t in threads:
        t.join(30)
    if any(t.is_alive() for t in threads):
        return {"algo": algo, "n": n, "dtype": str(dtype), "ok": False, "error": "timeout"}
    err = [e for e in errors if e]
    if err:
        return {"algo": algo, "n": n, "dtype": str(dtype), "ok": False, "error": err[0]}
    bad = []
    for r in range(P):
        for i in range(k):
            got = bufs[r][i].cpu().to(torch.int64)
            if not torch.equal(got, expect):
                bad.append([r, i, int((got != expect).sum())])
    return {"algo": algo, "n": n, "dtype": str(dtype).replace("torch.", ""), "ok": not bad,
            "mismatches": bad, "s": round(time.time() - t0, 3)}


def main():
    import torch
    ndev = torch.cuda.device_count()
    if SAME_DEVICE:
        ndev = 3
    elif ndev < 2:
        print(json.dumps({"devices": ndev, "ok": None, "skipped": "fewer than 2 GPUs"}))
        return 0
    import gloo_amd
    k = min(ndev, 4)
    cases = []
    for algo in ("ring_chunked", "halving_doubling"):
        for n, dtype in ((1000, torch.float32), ((1 << 20) + 3, torch.float32),
                         (100003, torch.int32)):
            cases.append(run_case(torch, gloo_amd, algo, k, n, dtype, seed=len(cases)))
            if cases[-1].get("error") == "timeout":  # rank threads still hold the GPUs
                break
        if cases and cases[-1].get("error") == "timeout":
            break
    print(json.dumps({"devices": k, "ok": all(c["ok"] for c in cases), "cases": cases,
                      "what": "2 thread-ranks x %d pointers on devices 0..%d; ring_chunked and "
                              "halving_doubling; integer-valued inputs, exact vs torch" % (k, k - 1)}))
    return 0


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    sys.exit(main())
