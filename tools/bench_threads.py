#!/usr/bin/env python3
"""Allreduce with P thread-ranks sharing ONE GPU (the reference's test
topology).  The peer copies are intra-device here, so the numbers bound the
protocol/executor overhead (host progress loop, events, credits, kernel
launches), not xGMI.  Prints one JSON line per (algo, P, elements).

    python tools/bench_threads.py [--P 2,4,8] [--elems 1024,...] [--iters 20]
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
    ap.add_argument("--P", default="2,4,8")
    ap.add_argument("--elems", default="1024,16384,262144,1048576,4194304,16777216,67108864")
    ap.add_argument("--algos", default="ring_chunked,ring_chunked_mesh,ring_chunked_repl,"
                                       "halving_doubling")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    import torch
    import gloo_amd
    for algo in args.algos.split(","):
        def cls(ctx, bufs_, algo=algo):
            if algo == "halving_doubling":
                return gloo_amd.AllreduceHalvingDoubling(ctx, bufs_)
            sched = {"ring_chunked_mesh": "mesh", "ring_chunked_repl": "replicated"}.get(
                algo, "ring")
            return gloo_amd.AllreduceRingChunked(ctx, bufs_, schedule=sched)
        for P in [int(x) for x in args.P.split(",")]:
            for n in [int(x) for x in args.elems.split(",")]:
                iters = args.iters if n <= (1 << 22) else max(3, args.iters // 4)
                bufs = [torch.rand(n, device="cuda") for _ in range(P)]
                torch.cuda.synchronize()
                store = gloo_amd.rendezvous.HashStore()
                times = [0.0] * P
                barrier = threading.Barrier(P)
                errs = []

                def rank(r):
                    try:
                        ctx = gloo_amd.rendezvous.Context(r, P, 0)
                        ctx.connectFullMesh(store)
                        alg = cls(ctx, [bufs[r]])
                        for _ in range(args.warmup):
                            alg.run()
                        barrier.wait()
                        t0 = time.perf_counter()
                        for _ in range(iters):
                            alg.run()
                        times[r] = time.perf_counter() - t0
                        barrier.wait()
                        alg.close()
                    except BaseException as e:  # noqa: BLE001
                        errs.append(repr(e))
                        try:
                            barrier.abort()
                        except Exception:  # noqa: BLE001
                            pass

                ts = [threading.Thread(target=rank, args=(r,)) for r in range(P)]
                [t.start() for t in ts]
                [t.join(300) for t in ts]
                if errs:
                    print(json.dumps({"algo": algo, "P": P, "elems": n, "error": errs[0]}))
                    continue
                t = max(times) / iters
                S = 4 * n
                print(json.dumps({"algo": algo, "P": P, "elems": n, "bytes": S,
                                  "us_per_op": round(t * 1e6, 1),
                                  "algbw_GBps": round(S / t / 1e9, 3)}), flush=True)
                del bufs


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
