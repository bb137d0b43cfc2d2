#!/usr/bin/env python3
"""Per-step cost of the device engines, measured on one GPU (ranks sharing
it, one hardware queue each): the ring on the plan kernel, the mesh on the
two-shot kernel and the replicated one-shot, from 1K to 64M fp32 elements
per rank.  With tiny buffers a run is almost all synchronisation: the ring's
time over its 4P-4 dependent sends bounds the per-step flag hand-off the
DESIGN.md 5b model charges.  One process per rank (launch with
tools/mp_launch.py --nproc P -- tools/scratch/step_latency.py); rank 0 prints
one JSON line.  GLOO_AMD_DEVTRACE=1 adds the kernels' own per-step traces
(stderr) for one run per size."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    import gloo_amd
    store = gloo_amd.rendezvous.PrefixStore(
        "steplat", gloo_amd.rendezvous.TorchStore(dist.distributed_c10d._get_default_store()))
    ctx = gloo_amd.rendezvous.Context(rank, world, 0)
    ctx.setTimeout(30)
    ctx.connectFullMesh(store)
    out = {"P": world, "queues": os.environ.get("GPU_MAX_HW_QUEUES", "4"), "us": {}}
    for n in (1 << 10, 1 << 14, 1 << 18, 1 << 22, 1 << 26):
        row = {}
        for sched in ("ring", "mesh", "replicated"):
            if sched == "replicated" and n > (1 << 20):
                continue
            buf = torch.ones(n, device="cuda")
            gloo_amd.set_steps_engine("device")
            alg = gloo_amd.AllreduceRingChunked(ctx, [buf], schedule=sched)
            gloo_amd.set_steps_engine("auto")
            for _ in range(3):
                alg.run()
            iters = 50 if n <= (1 << 18) else 10
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                alg.run()
            dt = torch.tensor([(time.perf_counter() - t0) / iters])
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            row[sched] = {"us": round(dt.item() * 1e6, 1), "engine": alg.engine()}
            alg.close()
            del buf
        out["us"][str(n)] = row
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
