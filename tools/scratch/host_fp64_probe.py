"""Probe: host-memory multi-pointer allreduce variants, mismatch ranges."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gloo_amd  # noqa: E402
from helpers import case_inputs, run_ranks  # noqa: E402
from oracle import oracle as O  # noqa: E402

TV = {O.FLOAT32: torch.float32, O.INT32: torch.int32, O.FLOAT16: torch.float16,
      O.FLOAT64: torch.float64}
FN = {O.SUM: "sum", O.PRODUCT: "product", O.MAX: "max"}


def run(P, N, dtype, op, nptrs, pinned, runs, algo="ring"):
    ins = case_inputs(P, N, dtype, nptrs, 0, seed=4)
    store = gloo_amd.rendezvous.HashStore()
    if pinned:
        bufs = [[torch.from_numpy(x.copy()).view(TV[dtype]).pin_memory() for x in row]
                for row in ins]
    else:
        bufs = [[np.array(x, copy=True) for x in row] for row in ins]
    engines = {}

    def rank_fn(r):
        ctx = gloo_amd.rendezvous.Context(r, P, 0)
        ctx.setTimeout(60)
        ctx.connectFullMesh(store)
        fn = getattr(gloo_amd.ReductionFunction, FN[op])
        if algo == "hd":
            alg = gloo_amd.AllreduceHalvingDoubling(ctx, bufs[r], fn=fn)
        else:
            alg = gloo_amd.AllreduceRingChunked(ctx, bufs[r], fn=fn, schedule="ring")
        engines[r] = alg.engine()
        for k in range(runs):
            if k > 0:
                for b, x in zip(bufs[r], ins[r]):
                    if pinned:
                        b.copy_(torch.from_numpy(x.copy()).view(b.dtype))
                    else:
                        b[...] = x
            alg.run()
        alg.close()
        return True

    run_ranks(P, rank_fn, timeout=120)
    code = O.HALVING_DOUBLING if algo == "hd" else O.RING_CHUNKED
    exp = O.allreduce(code, op, dtype, ins)
    bad = []
    for r in range(P):
        for i in range(nptrs):
            b = bufs[r][i]
            got = (b.view(torch.uint8).numpy().view(O.NP_DTYPE[dtype]) if pinned else b)
            e = exp[r][i]
            diff = np.nonzero((got.view(np.uint8).reshape(N, -1) !=
                               e.view(np.uint8).reshape(N, -1)).any(axis=1))[0]
            if diff.size:
                # contiguous ranges
                starts = [diff[0]]
                ends = []
                for a, c in zip(diff[:-1], diff[1:]):
                    if c != a + 1:
                        ends.append(a + 1)
                        starts.append(c)
                ends.append(diff[-1] + 1)
                rng = list(zip(starts, ends))[:6]
                bad.append((r, i, int(diff.size), rng))
    print("P %d N %d dtype %s op %s nptrs %d pinned %d runs %d algo %s engine %s: %s" % (
        P, N, O.DTYPE_NAMES[dtype], O.OP_NAMES[op], nptrs, pinned, runs, algo, engines.get(0),
        "OK" if not bad else "BAD %s" % bad[:4]), flush=True)


if __name__ == "__main__":
    for args in [
        (3, 300007, O.FLOAT64, O.PRODUCT, 2, 1, 2),
        (3, 300007, O.FLOAT64, O.PRODUCT, 2, 1, 1),
        (3, 300007, O.FLOAT64, O.PRODUCT, 1, 1, 1),
        (3, 300007, O.FLOAT64, O.SUM, 2, 1, 1),
        (3, 300007, O.FLOAT64, O.PRODUCT, 2, 0, 1),
        (3, 300007, O.FLOAT32, O.PRODUCT, 2, 1, 1),
        (3, 600007, O.FLOAT32, O.PRODUCT, 2, 1, 1),
        (3, 300007, O.INT32, O.SUM, 2, 1, 1),
        (3, 600007, O.INT32, O.SUM, 2, 1, 1),
        (2, 300007, O.FLOAT64, O.SUM, 1, 0, 1),
        (3, 300007, O.FLOAT64, O.PRODUCT, 2, 1, 1, "hd"),
    ]:
        run(*args)
