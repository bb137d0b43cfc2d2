#!/usr/bin/env python3
"""The host-issued ring's hand-off cost per dependent round without
processes sharing the GPU: P rank THREADS of one process on the box's GPU
(the reference tests' topology, gloo/test/base_test.h:91-166), schedule
"ring", host-issued steps (the only engine for threads sharing a device),
at sizes where the bytes cost next to nothing.  tools/hop_latency.py runs
the same ring with one process per rank; on one GPU those processes'
kernels and copies interleave through the GPU's queues, which this
variant avoids.  Prints one JSON line: us per allreduce (slowest rank) and
per round (2 (P - 1) rounds).

    python tools/hop_latency_threads.py [--ranks 2,4,8] [--sizes 1024,65536]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--sizes", default="1024,65536,1048576")
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    import torch

    import gloo_amd
    out = {}
    for P in [int(x) for x in a.ranks.split(",")]:
        row = {}
        for n in [int(x) for x in a.sizes.split(",")]:
            store = gloo_amd.rendezvous.HashStore()
            bufs = [torch.zeros(n, dtype=torch.float32, device="cuda") for _ in range(P)]
            torch.cuda.synchronize()
            times = [0.0] * P
            engines = [None] * P
            errors = []
            barrier = threading.Barrier(P)

            def rank(r):
                try:
                    ctx = gloo_amd.rendezvous.Context(r, P, 0)
                    ctx.connectFullMesh(store)
                    alg = gloo_amd.AllreduceRingChunked(ctx, [bufs[r]], schedule="ring")
                    engines[r] = alg.engine()
                    for _ in range(10):
                        alg.run()
                    barrier.wait()
                    t0 = time.perf_counter()
                    for _ in range(a.iters):
                        alg.run()
                    times[r] = time.perf_counter() - t0
                    barrier.wait()
                    alg.close()
                    ctx.close()
                except BaseException as e:  # noqa: BLE001
                    errors.append(repr(e))
                    barrier.abort()
            ts = [threading.Thread(target=rank, args=(r,)) for r in range(P)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            if errors:
                row[str(n)] = {"error": errors[0][:300]}
                continue
            us = max(times) / a.iters * 1e6
            row[str(n)] = {"engine": engines[0], "us_per_allreduce": round(us, 2),
                           "us_per_round": round(us / (2 * (P - 1)), 2),
                           "result_ok": all(bool((b == 0).all().item()) for b in bufs)}
        out["P%d" % P] = row
    print(json.dumps({"what": "ring (schedule=ring), P rank threads of one process on one GPU, "
                              "host-issued steps; us per allreduce (slowest rank) and per "
                              "dependent round", "iters": a.iters, "results": out}), flush=True)


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
