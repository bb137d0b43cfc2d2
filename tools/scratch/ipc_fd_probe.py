"""How many file descriptors does each algorithm instance cost a rank, and do
they come back on close?  (IPC in dmabuf mode passes file descriptors.)  One
process per rank:

    python tools/mp_launch.py --nproc P -- tools/ipc_fd_probe.py DIR
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def nfd():
    return len(os.listdir("/proc/self/fd"))


def main():
    import resource

    import torch

    import gloo_amd

    rank, size = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    store = gloo_amd.rendezvous.FileStore(sys.argv[1])
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(30)
    ctx.connectFullMesh(store)
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    print("r%d fd limit soft %d hard %d; open after connect %d" % (rank, soft, hard, nfd()),
          flush=True)
    buf = torch.ones(1 << 20, device="cuda")
    torch.cuda.synchronize()
    kinds = [("repl", dict(schedule="replicated")), ("mesh", dict(schedule="mesh")),
             ("ring", dict(schedule="ring"))]
    for it in range(30):
        for name, kw in kinds:
            before = nfd()
            try:
                alg = gloo_amd.AllreduceRingChunked(ctx, [buf], **kw)
                alg.run()
                during = nfd()
                eng = alg.engine()
                alg.close()
            except Exception as e:  # noqa: BLE001 - report and stop
                print("r%d iter %d %s FAILED with %d fds open: %s" % (rank, it, name, nfd(), e),
                      flush=True)
                sys.exit(1)
            if it < 2 or it % 10 == 0:
                print("r%d iter %d %s (%s): fds %d -> %d -> %d" % (rank, it, name, eng, before,
                                                                    during, nfd()), flush=True)
    print("r%d OK, %d fds open at the end" % (rank, nfd()), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
