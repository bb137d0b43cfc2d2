"""One rank of the multi-process GPU test (tests/test_allreduce_gpu.py).

    python mp_worker.py <store_dir> <rank> <size> <algo>

algo: ring_chunked | halving_doubling | ring_chunked_mesh (class algorithms)
      fn_ring | fn_bcube | fn_ring_mesh (gloo_amd.allreduce, two calls with
      different buffers, the second out of place)

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
    if algo.startswith("fn_"):
        return run_fn(store_dir, rank, size, algo, N)
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


def run_fn(store_dir, rank, size, algo, N):
    import numpy as np
    import torch

    import gloo_amd
    from helpers import case_inputs
    from oracle import oracle as O

    code = {"fn_ring": 1, "fn_bcube": 2, "fn_ring_mesh": 3}[algo]
    data = case_inputs(size, N, O.FLOAT32, 1, 0, seed=33)
    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(60)
    ctx.connectFullMesh(store)
    # call 1: in place
    out = torch.from_numpy(data[rank][0].copy()).cuda()
    opts = gloo_amd.AllreduceOptions(ctx)
    opts.setAlgorithm(code)
    opts.setOutput(out)
    opts.setReduceFunction(gloo_amd.ReductionFunction.sum)
    gloo_amd.allreduce(opts)
    ocode = O.FN_BCUBE if code == 2 else O.FN_RING
    exp = O.allreduce_fn(ocode, O.SUM, O.FLOAT32, [[] for _ in range(size)], data)[rank][0]
    ok = np.array_equal(out.cpu().numpy().view(np.uint32), exp.view(np.uint32))
    # call 2: out of place into a new buffer (the cached executor is reused)
    inp = torch.from_numpy(data[rank][0].copy()).cuda()
    out2 = torch.zeros(N, device="cuda")
    opts = gloo_amd.AllreduceOptions(ctx)
    opts.setAlgorithm(code)
    opts.setInput(inp)
    opts.setOutput(out2)
    opts.setReduceFunction(gloo_amd.ReductionFunction.sum)
    gloo_amd.allreduce(opts)
    ok = ok and np.array_equal(out2.cpu().numpy().view(np.uint32), exp.view(np.uint32))
    store.set("done/%d" % rank, b"1")
    for r in range(size):
        store.get("done/%d" % r, timeout_ms=60000)
    ctx.close()
    if not ok:
        print("MISMATCH rank", rank)
        sys.exit(1)
    print("OK")


if __name__ == "__main__":
    main()
