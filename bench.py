#!/usr/bin/env python3
"""Benchmark of the MI355X gloo allreduce hot path (BASELINE.json metric:
"allreduce GB/s (device-resident, fp32) at 1/2/4/8 MI355X; % HBM|xGMI roofline").

  python bench.py [--gpus 1] [--steps K] [--warmup W]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
      --master-addr 127.0.0.1 --master-port P bench.py --gpus N

N == 1  -> workload = BASELINE configs[1]: local reduce (sum) of one 256 MiB
           fp32 buffer on one MI355X: c = a + b with the glx reduce kernel.
           A step = one kernel pass over the 256 MiB.
N  > 1  -> workload = configs[2]/north star: allreduce_ring_chunked of a
           256 MiB fp32 buffer per rank, one process per GPU, chunks moved
           over xGMI with hipMemcpyPeerAsync.  A step = one run().
value   = whole-job bytes reduced per second = N * S / t_step (GB/s, 1e9),
           S = 256 MiB per rank, t_step from the max over ranks.
Inputs are synthetic, resident in HBM before the timed region.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0     # MI355X spec (MI355X_MICROARCH.md)
XGMI_LINK_GBPS = 153.0     # per link, per direction (task statement)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--size-mib", type=int, default=256)
    p.add_argument("--algo", default="ring_chunked",
                   choices=["ring_chunked", "halving_doubling", "ring_chunked_mesh"])
    p.add_argument("--no-alt", action="store_true",
                   help="N>1: do not also time the other schedules")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="bounded CPU baseline sample (seconds of CPU work)")
    p.add_argument("--kernel-only", action="store_true",
                   help="N=1: run only the timed kernel loop (for rocprofv3 --pmc)")
    return p.parse_args()


def load_traffic(workload):
    """HBM bytes per launch from a PMC pass (profiles/*_pmc_traffic.json,
    written by tools/pmc_traffic.py from rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE, FETCH_SIZE doubled per the gfx950 correction)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(workload, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(nbytes, seconds):
    """gloo::sum<float> on the host cores (single thread, like the reference):
    the reference itself (oracle/_ref, compiled from the reference sources in
    the build container) when present, else the oracle's restatement."""
    import numpy as np
    from oracle import oracle as O
    n = nbytes // 4
    a = O.fill(O.FLOAT32, n, 0, seed=1234, rank=0)
    b = O.fill(O.FLOAT32, n, 0, seed=1234, rank=1)
    c = np.empty_like(a)
    kind = "reference" if O.ref_available() else "port"
    if kind == "reference":
        lib = O._load_ref()

        def step():
            lib.ref_reduce(O.SUM, O.FLOAT32, O._ptr(c), O._ptr(a), O._ptr(b), n)
    else:
        def step():
            O.sum_f32(c, a, b)
    step()  # page in
    reps, t0 = 0, time.perf_counter()
    while True:
        step()
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds or reps >= 2000:
            break
    t = el / reps
    return {"value": round(nbytes / t / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": kind,
            "sample": "gloo::sum<float> c=a+b over %d MiB, %d reps in %.1f s, 1 thread "
                      "(%s)" % (nbytes >> 20, reps, el,
                                "oracle/_ref: reference gloo/math.h" if kind == "reference"
                                else "oracle port of gloo/math.h"),
            "ms_per_step": round(t * 1e3, 3), "nproc": os.cpu_count()}


def bench_single(args):
    import torch
    import gloo_amd
    S = args.size_mib << 20
    n = S // 4
    steps = args.steps or 100
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1234)
    a = torch.rand(n, device=dev, generator=g) * 2 - 1
    b = torch.rand(n, device=dev, generator=g) * 2 - 1
    c = torch.empty_like(a)
    stream = torch.cuda.current_stream(dev)
    for _ in range(args.warmup):
        gloo_amd.math.sum(c, a, b, stream=stream)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)  # the kernels are launched on this stream
    for _ in range(steps):
        gloo_amd.math.sum(c, a, b, stream=stream)
    ev1.record(stream)
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / steps
    if args.kernel_only:
        return None
    ok = bool(torch.equal(c, a + b))
    t = ms / 1e3
    alg_bytes = 3 * S  # two reads + one write per launch
    achieved = alg_bytes / t / 1e9
    workload = "local_reduce_sum_fp32_256MiB"
    traffic = load_traffic(workload)
    res = {
        "metric": "allreduce GB/s (device-resident, fp32) at 1/2/4/8 MI355X; % HBM|xGMI roofline",
        "value": round(S / t / 1e9, 3), "unit": "GB/s", "n_gpus": 1, "steps": steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 5), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": workload, "bytes_per_rank": S, "elements": n,
                   "op": "sum", "kernel": "glx reduce_kernel<float,SUM> (HIP, gfx950)",
                   "baseline_config": "configs[1]"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": traffic,
                     "algorithmic_bytes_per_launch": alg_bytes},
        "verified": ok,
    }
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(S, args.cpu_seconds)
    return res


def reduce_kernel_roofline(torch, gloo_amd, dev, chunk_bytes, reps=50):
    """Live HBM roofline of the reduce kernel at the ring's chunk size, timed
    with HIP events on the stream it is launched on."""
    n = chunk_bytes // 4
    a = torch.rand(n, device=dev)
    b = torch.rand(n, device=dev)
    s = torch.cuda.current_stream(dev)
    for _ in range(5):
        gloo_amd.math.reduce(gloo_amd.ReductionType.SUM, a, a, b, stream=s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        gloo_amd.math.reduce(gloo_amd.ReductionType.SUM, a, a, b, stream=s)
    e1.record(s)
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / reps / 1e3
    ach = 3 * chunk_bytes / t / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": None,
            "kernel": "reduce in place, %d MiB chunk" % (chunk_bytes >> 20),
            "algorithmic_bytes_per_launch": 3 * chunk_bytes}


def make_alg(gloo_amd, ctx, buf, algo):
    if algo == "halving_doubling":
        return gloo_amd.AllreduceHalvingDoubling(ctx, [buf])
    return gloo_amd.AllreduceRingChunked(ctx, [buf],
                                        schedule="mesh" if algo == "ring_chunked_mesh" else "ring")


def time_schedule(torch, dist, gloo_amd, ctx, buf, algo, steps, warmup):
    """warmup untimed runs, then `steps` timed runs between barriers +
    device syncs; returns (max-over-ranks seconds per step, link bytes/run)."""
    alg = make_alg(gloo_amd, ctx, buf, algo)
    for _ in range(warmup):
        alg.run()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        alg.run()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    dist.barrier()
    el = torch.tensor([t1 - t0], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    sent = alg.bytes_sent()
    alg.close()
    return el.item() / steps, sent


def bench_multi(args):
    import torch
    import torch.distributed as dist
    import gloo_amd
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    # one GPU per rank; on a box with fewer GPUs than ranks (rehearsal only)
    # ranks share devices round-robin
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("gloo")  # host-side coordination only
    S = args.size_mib << 20
    n = S // 4
    steps = args.steps or 20
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    src = torch.rand(n, device=dev, generator=g) * 2 - 1
    buf = src.clone()
    torch.cuda.synchronize()
    store = gloo_amd.rendezvous.PrefixStore(
        "gloo_amd_bench", gloo_amd.rendezvous.TorchStore(dist.distributed_c10d._get_default_store()))
    ctx = gloo_amd.rendezvous.Context(rank, world, local)
    ctx.setTimeout(120)
    ctx.connectFullMesh(store)
    t, link_bytes = time_schedule(torch, dist, gloo_amd, ctx, buf, args.algo, steps,
                                  args.warmup)
    # correctness after the timing: one more run on fresh inputs; every rank
    # must hold the same bits (the reduction order is rank-independent)
    buf.copy_(src)
    torch.cuda.synchronize()
    alg = make_alg(gloo_amd, ctx, buf, args.algo)
    alg.run()
    torch.cuda.synchronize()
    alg.close()
    cs = torch.tensor([int(buf.view(torch.int32).to(torch.int64).sum().item())],
                      dtype=torch.int64)
    allcs = [torch.zeros_like(cs) for _ in range(world)]
    dist.all_gather(allcs, cs)
    verified = all(int(x.item()) == int(cs.item()) for x in allcs)
    alts = {}
    if not args.no_alt:
        for other in ("ring_chunked", "ring_chunked_mesh", "halving_doubling"):
            if other == args.algo:
                continue
            buf.copy_(src)
            torch.cuda.synchronize()
            ta, sent_a = time_schedule(torch, dist, gloo_amd, ctx, buf, other, steps,
                                       args.warmup)
            alts[other] = {"value": round(world * S / ta / 1e9, 3),
                           "ms_per_step": round(ta * 1e3, 4),
                           "algbw_GBps": round(S / ta / 1e9, 3),
                           "link_bytes_per_step": sent_a}
    res = None
    if rank == 0:
        chunk = max(256 * 4, -(-S // (2 * world)))
        algbw = S / t / 1e9
        busbw = algbw * 2 * (world - 1) / world
        link_ach = link_bytes / t / 1e9
        res = {
            "metric": "allreduce GB/s (device-resident, fp32) at 1/2/4/8 MI355X; % HBM|xGMI roofline",
            "value": round(world * S / t / 1e9, 3), "unit": "GB/s", "n_gpus": world,
            "steps": steps, "warmup": args.warmup, "ms_per_step": round(t * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic",
            "config": {"workload": "allreduce_%s_fp32_256MiB_per_rank" % args.algo,
                       "algorithm": args.algo, "bytes_per_rank": S, "elements": n,
                       "parallelism": "dp%d" % world, "transport": "hipMemcpyPeerAsync/xGMI",
                       "baseline_config": "configs[3]" if args.algo == "halving_doubling"
                       else "configs[2]"},
            "algbw_GBps": round(algbw, 3), "busbw_GBps": round(busbw, 3),
            "roofline": reduce_kernel_roofline(torch, gloo_amd, dev, chunk),
            "link_roofline": {"bound": "xgmi_link", "achieved": round(link_ach, 2),
                              "peak": XGMI_LINK_GBPS, "unit": "GB/s",
                              "frac": round(link_ach / XGMI_LINK_GBPS, 4),
                              "link_bytes_per_step": link_bytes,
                              "note": "bytes this rank sent per step / step time; the "
                                      "ring uses one link per direction"},
            "alt_schedules": alts,
            "verified": verified,
        }
    dist.barrier()
    dist.destroy_process_group()
    return res


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        res = bench_multi(args)
    else:
        if args.gpus > 1:
            sys.exit("bench.py --gpus N>1 must be launched with torch.distributed.run "
                     "(one process per GPU)")
        res = bench_single(args)
    if res is not None:
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
