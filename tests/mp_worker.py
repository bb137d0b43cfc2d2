"""One rank of the multi-process GPU test (tests/test_allreduce_gpu.py).

    python mp_worker.py <store_dir> <rank> <size> <ring_chunked|halving_doubling>

Checks its result against the oracle and prints OK."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def main():
    store_dir, rank, size, algo = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    import numpy as np
    import torch

    import gloo_amd
    from helpers import case_inputs
    from oracle import oracle as O

    N = 100003
    code = O.HALVING_DOUBLING if algo == "halving_doubling" else O.RING_CHUNKED
    ins = case_inputs(size, N, O.FLOAT32, 1, 0, seed=31)
    buf = torch.from_numpy(ins[rank][0].copy()).cuda()
    torch.cuda.synchronize()
    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(60)
    ctx.connectFullMesh(store)
    if algo == "halving_doubling":
        alg = gloo_amd.AllreduceHalvingDoubling(ctx, [buf])
    else:
        alg = gloo_amd.AllreduceRingChunked(
            ctx, [buf], schedule="mesh" if algo == "ring_chunked_mesh" else "ring")
    for _ in range(2):
        buf.copy_(torch.from_numpy(ins[rank][0].copy()).cuda())
        torch.cuda.synchronize()
        alg.run()
    exp = O.allreduce(code, O.SUM, O.FLOAT32, ins)[rank][0]
    got = buf.cpu().numpy()
    if not np.array_equal(got.view(np.uint32), exp.view(np.uint32)):
        bad = np.nonzero(got != exp)[0]
        print("MISMATCH rank", rank, "count", bad.size, "first", bad[:8])
        sys.exit(1)
    # keep the process (and its receive regions) alive until every rank is done
    store.set("done/%d" % rank, b"1")
    for r in range(size):
        store.get("done/%d" % r, timeout_ms=60000)
    alg.close()
    print("OK")


if __name__ == "__main__":
    main()
