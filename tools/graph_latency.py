#!/usr/bin/env python3
"""Small-message allreduce latency, eager vs HIP graph: one
process per rank (torchrun or tools/mp_launch.py), each with its device
engine on a caller's stream.  Eager: `iters` run() calls back to back on the
stream, one synchronize at the end.  Graph: `per_graph` run() calls captured
into one torch.cuda.CUDAGraph, replayed iters / per_graph times.  Reports
microseconds per allreduce (max over ranks), per size and schedule, as one
JSON line on rank 0.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        tools/graph_latency.py [--sizes 256,4096,65536] [--iters 400]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="256,4096,65536,1048576")
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--per-graph", type=int, default=20)
    ap.add_argument("--schedules", default="replicated,ring,fn_replicated,fn_ring")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    import gloo_amd
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    ctx = gloo_amd.rendezvous.Context(rank, world, dev)
    ctx.connectFullMesh(gloo_amd.rendezvous.TorchStore(dist.distributed_c10d._get_default_store()))
    s = torch.cuda.Stream()
    out = {}

    def timed(fn, n):
        """(seconds for n calls including the GPU's, seconds to issue them),
        each the max over ranks"""
        s.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        fn(n)
        t1 = time.perf_counter()
        s.synchronize()
        el = torch.tensor([time.perf_counter() - t0, t1 - t0], dtype=torch.float64)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return el[0].item(), el[1].item()

    for idx, n in enumerate([int(x) for x in a.sizes.split(",")]):
        key = str(n) if str(n) not in out else "%d#%d" % (n, idx)  # a size again
        for sched in [x for x in a.schedules.split(",") if not x.startswith("fn_")]:
            buf = torch.zeros(n, dtype=torch.float32, device="cuda")
            alg = gloo_amd.AllreduceRingChunked(ctx, [buf], streams=[s], schedule=sched)
            engine = alg.engine()
            if engine == "steps":  # host-issued steps wait on the host: not capturable
                alg.close()
                continue
            for _ in range(5):
                alg.run()

            def eager(k):
                for _ in range(k):
                    alg.run()
            eager_s, issue_s = timed(eager, a.iters)
            g = torch.cuda.CUDAGraph()
            s.synchronize()
            with torch.cuda.graph(g, stream=s):
                for _ in range(a.per_graph):
                    alg.run()

            def replay(k):
                with torch.cuda.stream(s):
                    for _ in range(k // a.per_graph):
                        g.replay()
            graph_s = timed(replay, a.iters)[0]
            s.synchronize()
            ok = bool((buf == 0).all().item())  # zeros stay zeros, run after run
            del g
            alg.close()
            out.setdefault(key, {})[sched] = {
                "engine": engine, "eager_us": round(eager_s / a.iters * 1e6, 2),
                "eager_issue_us": round(issue_s / a.iters * 1e6, 2),
                "graph_us": round(graph_s / (a.iters // a.per_graph * a.per_graph) * 1e6, 2),
                "result_ok": ok}
        # the function-style call (gloo::allreduce(opts)) on the same stream,
        # eager only: its executor comes from a cache keyed by the call
        fns = {"fn_replicated": gloo_amd.AllreduceOptions.Algorithm.RING_REPLICATED,
               "fn_ring": gloo_amd.AllreduceOptions.Algorithm.RING}
        for name in [x for x in a.schedules.split(",") if x.startswith("fn_")]:
            algo = fns[name]
            buf = torch.zeros(n, dtype=torch.float32, device="cuda")
            opts = gloo_amd.AllreduceOptions(ctx)
            opts.setAlgorithm(algo)
            opts.setOutput(buf)
            opts.setStream(s)
            for _ in range(5):
                gloo_amd.allreduce(opts)

            def fn_calls(k):
                for _ in range(k):
                    gloo_amd.allreduce(opts)
            fn_s, fn_issue_s = timed(fn_calls, a.iters)
            again_s = timed(fn_calls, a.iters)[0]  # a one-time cost shows as a gap
            s.synchronize()
            out.setdefault(key, {})[name] = {
                "eager_us": round(fn_s / a.iters * 1e6, 2),
                "eager_again_us": round(again_s / a.iters * 1e6, 2),
                "eager_issue_us": round(fn_issue_s / a.iters * 1e6, 2),
                "result_ok": bool((buf == 0).all().item())}
    # the floor for a kernel launched from Python on the same stream: a
    # torch elementwise op of the smallest size, back to back
    x = torch.zeros(256, dtype=torch.float32, device="cuda")

    def torch_op(k):
        with torch.cuda.stream(s):
            for _ in range(k):
                x.add_(0.0)
    torch_op(20)  # loads the op's code object
    op_s, op_issue_s = timed(torch_op, a.iters)
    if rank == 0:
        print(json.dumps({"what": "allreduce latency per call, eager (back to back on a stream) "
                                  "vs HIP graph replay (%d calls per graph), max over ranks"
                                  % a.per_graph, "ranks": world, "sizes": out,
                          "torch_add_us": round(op_s / a.iters * 1e6, 2),
                          "torch_add_issue_us": round(op_issue_s / a.iters * 1e6, 2)}))
    dist.barrier()
    ctx.close()


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
