#!/usr/bin/env python3
"""Create / run / close churn of rank THREADS in one process (the shape of
tools/hop_latency_threads.py, whose first run died once with SIGSEGV --
DESIGN.md 9): rounds of P = 2, 4, 8 thread-ranks, each building a context
and a ring_chunked algorithm on the box's GPU, running it, then closing the
algorithm and the context at once, with no barrier between the ranks'
closes.  Prints a progress line per round (flushed), so a crash names the
round it happened in; run it under `python -X faulthandler` for the stacks.

    python -X faulthandler tools/stress_threads.py [--rounds 30]
"""
import argparse
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--runs", type=int, default=50)
    ap.add_argument("--close", default="explicit", choices=["explicit", "gc"],
                    help="explicit: each rank closes its algorithm and context at once; "
                         "gc: each rank drops them and the garbage collector destroys the "
                         "native handles from whichever thread runs it")
    a = ap.parse_args()
    import gc
    import torch

    import gloo_amd
    t0 = time.time()
    for it in range(a.rounds):
        for P in (2, 4, 8):
            n = (1024, 65536, 1 << 20)[it % 3]
            store = gloo_amd.rendezvous.HashStore()
            bufs = [torch.full((n,), float(r), device="cuda") for r in range(P)]
            torch.cuda.synchronize()
            errors = []

            def rank(r):
                try:
                    ctx = gloo_amd.rendezvous.Context(r, P, 0)
                    ctx.connectFullMesh(store)
                    alg = gloo_amd.AllreduceRingChunked(ctx, [bufs[r]], schedule="ring")
                    for _ in range(a.runs):
                        alg.run()
                    if a.close == "explicit":
                        alg.close()
                        ctx.close()
                    else:
                        del alg, ctx  # __del__ (Algorithm, Context) wherever GC runs
                except BaseException as e:  # noqa: BLE001
                    errors.append(repr(e)[:300])
            ts = [threading.Thread(target=rank, args=(r,)) for r in range(P)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            gc.collect()
            # the runs fold the values again and again: only the bits'
            # agreement across ranks is checked
            same = all(torch.equal(bufs[0], b) for b in bufs[1:])
            print("round %d P %d n %d errors %d same %s t %.1f s" % (
                it, P, n, len(errors), same, time.time() - t0), flush=True)
            if errors or not same:
                print("FAIL", errors[:2], flush=True)
                return 1
    print("OK", flush=True)
    return 0


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    sys.exit(main())
