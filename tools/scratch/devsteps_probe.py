"""Diagnose first-run mismatches of the plan kernel (engine devsteps) with
many ranks: runs the worker's dtype cases, reports per run how many elements
differ from the oracle and where, optionally with a store barrier before
every close (CLOSE_BARRIER=1).  One process per rank:

    python tools/mp_launch.py --nproc 8 -- tools/scratch/devsteps_probe.py DIR
"""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))


def main():
    import time

    import numpy as np
    import torch

    import gloo_amd
    from helpers import case_inputs
    from oracle import oracle as O
    from test_reduce_gpu import from_dev, to_dev

    rank, size = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    barrier = os.environ.get("CLOSE_BARRIER") == "1"
    torch.cuda.set_device(0)
    store = gloo_amd.rendezvous.FileStore(sys.argv[1])
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(60)
    ctx.connectFullMesh(store)
    gloo_amd.set_steps_engine("device")
    # EXTRA_STREAMS=k: k more streams with a kernel each before the cases
    # (more hardware queues per process, as host-steps algorithms create)
    keep = []
    for _ in range(int(os.environ.get("EXTRA_STREAMS", "0"))):
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            keep.append(torch.ones(1024, device="cuda") * 2)
        keep.append(st)
    torch.cuda.synchronize()
    reps = int(os.environ.get("REPEAT", "1"))
    cases = []
    if os.environ.get("WITH_F32") == "1":  # the worker's f32 series first
        for n in (1, 3, 255, 256, 1000, 4099, 65539, 1 << 20, (1 << 22) + 5):
            cases.append((n, O.FLOAT32, O.SUM))
    for _ in range(reps):
        for dt in (O.FLOAT16, O.BFLOAT16, O.INT32, O.FLOAT64):
            for op in (O.SUM, O.PRODUCT, O.MAX, O.MIN):
                cases.append((4099, dt, op))
    nbad = 0
    for seed, (n, dt, op) in enumerate(cases):
        ins = case_inputs(size, n, dt, 1, 0, seed=300 + seed)
        exp = O.allreduce(O.RING_CHUNKED, op, dt, ins)[rank][0]
        buf = to_dev(ins[rank][0], dt)
        alg = gloo_amd.AllreduceRingChunked(ctx, [buf], fn=gloo_amd.ReductionFunction(op),
                                           schedule="ring", dtype=dt)
        for it in range(3):
            buf.copy_(to_dev(ins[rank][0], dt))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            alg.run()
            ms = (time.perf_counter() - t0) * 1e3
            if rank == 0:
                print("r0 case %d n %d dt %d op %d run %d engine %s %.2f ms"
                      % (seed, n, dt, op, it, alg.engine(), ms), flush=True)
            got = np.ascontiguousarray(from_dev(buf, dt)).view(np.uint8)
            ref = np.ascontiguousarray(exp).view(np.uint8)
            es = ref.size // n
            diff = np.nonzero((got.reshape(n, es) != ref.reshape(n, es)).any(axis=1))[0]
            if diff.size:
                nbad += 1
                inp = np.ascontiguousarray(ins[rank][0]).view(np.uint8).reshape(n, es)
                i = int(diff[0])
                print("r%d case %d dt %d op %d run %d engine %s: %d bad elems, first %d last %d;"
                      " at first got %s exp %s own-input %s"
                      % (rank, seed, dt, op, it, alg.engine(), diff.size, i, int(diff[-1]),
                         got.reshape(n, es)[i].tobytes().hex(), ref.reshape(n, es)[i].tobytes().hex(),
                         inp[i].tobytes().hex()), flush=True)
        if barrier:
            store.set("closebar/%d/%d" % (seed, rank), b"1")
            for r in range(size):
                store.get("closebar/%d/%d" % (seed, r), timeout_ms=60000)
        alg.close()
    print("r%d done, %d bad runs" % (rank, nbad), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
