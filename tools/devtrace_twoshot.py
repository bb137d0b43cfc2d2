"""Phase timing of the two-shot kernel (GLOO_AMD_DEVTRACE=1 makes the
executor print per-phase stamps after every launch).  One process per rank:

    GLOO_AMD_DEVTRACE=1 python tools/mp_launch.py --nproc 2 -- tools/devtrace_twoshot.py DIR
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import torch

    import gloo_amd

    rank, size = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    store = gloo_amd.rendezvous.FileStore(sys.argv[1])
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(30)
    ctx.connectFullMesh(store)
    for n in (1 << 10, 1 << 18, 1 << 20, 1 << 22, 1 << 24, 1 << 26):
        buf = torch.ones(n, device="cuda")
        torch.cuda.synchronize()
        alg = gloo_amd.AllreduceRingChunked(ctx, [buf], schedule="mesh")
        assert alg.engine() == "twoshot", alg.engine()
        print("r%d n=%d" % (rank, n), file=sys.stderr, flush=True)
        for _ in range(4):
            alg.run()
        alg.close()
    ctx.close()


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
