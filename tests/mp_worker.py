"""One rank of the multi-process GPU test (tests/test_allreduce_gpu.py).

    python mp_worker.py <store_dir> <rank> <size> <algo>

algo: ring_chunked | halving_doubling | ring_chunked_mesh (class algorithms)
      fn_ring | fn_bcube | fn_ring_mesh (gloo_amd.allreduce, two calls with
      different buffers, the second out of place)
      oneshot | twoshot (the replicated / mesh schedule as one device-driven
      kernel per rank: class and function style, dtypes x ops x sizes,
      device and host buffers, repeated runs; prints per-op latencies)
      devsteps (ring_chunked, halving_doubling, function-style ring and bcube
      through the plan kernel: dtypes x ops x sizes, device and host buffers,
      repeated runs; prints per-op latencies of the plan kernel vs the
      host-issued steps)
      dmasteps (the same cases through the DMA steps engine: the host-issued
      program's copies and reduce launches with on-GPU hand-offs)
      devtimeout (rank 0 runs the one- and two-shot kernels and the DMA steps
      engine while the other ranks never call run(): its kernels must give up
      after the timeout and run() must raise IoException)
      scale:cfg34 | scale:cfg5 (BASELINE.json configs at full size, 8 ranks:
      every engine's output SHA-256 against tests/golden/scale_golden.json)
      scale:ns (the north-star size, 256 MiB fp32 per rank, ring and HD at
      P = size: every engine against tests/golden/bench_golden.json)
      linkprobe (the measured-link probe through the product's IPC path, and
      every peer's connect-time view; then an allreduce on the same context)
      engine_choice (which engine the automatic policy picks on the shared
      GPU under this process's GPU_MAX_HW_QUEUES, and one exact run)
      fuzz:<seed> (randomized algorithms / lengths / dtypes / ops / host
      buffers on the device engines, every rank the same draw, each against
      the oracle)
      maxcount (the class algorithms at the largest count the reference's
      `const int count` takes, INT_MAX elements, int8 and float16, P = 2, on
      every engine: exact, the result must equal x0 + x1)
      big:fast | big:plain (the ring on the plan kernel over MORE than 2 GiB per
      rank, P = 2, the given stream policy: every 32-bit store offset the
      write-through path could form is exceeded; exact at P = 2 since fp32
      addition commutes: the result must equal x0 + x1 bit for bit)

Checks its result against the oracle and prints OK."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def main():
    import faulthandler
    faulthandler.enable()  # a crash of any rank prints its threads' stacks
    store_dir, rank, size, algo = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    import numpy as np
    import torch

    import gloo_amd
    from helpers import case_inputs
    from oracle import oracle as O

    N = 100003
    if algo in ("oneshot", "twoshot"):
        return run_device(store_dir, rank, size, algo)
    if algo == "devtimeout":
        return run_device_timeout(store_dir, rank, size)
    if algo == "dmaabort":
        return run_dma_abort(store_dir, rank, size)
    if algo == "custom":
        return run_custom(store_dir, rank, size)
    if algo == "class_custom":
        return run_class_custom(store_dir, rank, size)
    if algo.startswith("killpeer:"):
        return run_killpeer(store_dir, rank, size, *algo.split(":")[1:])
    if algo == "devsteps":
        return run_devsteps(store_dir, rank, size)
    if algo == "dmasteps":
        return run_devsteps(store_dir, rank, size, eng="dma")
    if algo == "churn":
        return run_churn(store_dir, rank, size)
    if algo.startswith("scale:"):
        return run_scale(store_dir, rank, size, algo[len("scale:"):])
    if algo.startswith("fuzz:"):
        return run_fuzz(store_dir, rank, size, int(algo[len("fuzz:"):]))
    if algo.startswith("graph:"):
        return run_graph(store_dir, rank, size, int(algo[len("graph:"):]))
    if algo.startswith("soak:"):
        parts = algo.split(":")
        return run_soak(store_dir, rank, size, int(parts[1]),
                        uneven=parts[2] if len(parts) > 2 else "",
                        n=int(parts[3]) if len(parts) > 3 and parts[3] else 1 << 20)
    if algo.startswith("big:"):
        return run_big(store_dir, rank, size, algo[len("big:"):])
    if algo == "maxcount":
        return run_maxcount(store_dir, rank, size)
    if algo == "linkprobe":
        return run_linkprobe(store_dir, rank, size)
    if algo.startswith("graph_overlap:"):
        parts = algo.split(":")
        return run_graph_overlap(store_dir, rank, size, parts[1],
                                 close_first=len(parts) > 2 and parts[2] == "close")
    if algo == "engine_choice":
        return run_engine_choice(store_dir, rank, size)
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


def run_device_timeout(store_dir, rank, size):
    import time

    import torch

    import gloo_amd

    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(3)
    ctx.connectFullMesh(store)
    ok = True
    for sched, eng, n in (("replicated", "oneshot", 4099), ("mesh", "twoshot", 1 << 20),
                          ("ring", "dmasteps", 1 << 20)):
        buf = torch.ones(n, device="cuda")
        gloo_amd.set_steps_engine("dma" if eng == "dmasteps" else "auto")
        try:
            alg = gloo_amd.AllreduceRingChunked(ctx, [buf], schedule=sched)
        finally:
            gloo_amd.set_steps_engine("auto")
        ok = ok and alg.engine() == eng
        if rank == 0:
            t0 = time.time()
            try:
                alg.run()
                print("NO TIMEOUT", sched)
                ok = False
            except gloo_amd.IoException as e:
                dt = time.time() - t0
                print("timed out as expected after %.1f s: %s" % (dt, e))
                ok = ok and "Timed out" in str(e) and dt < 30
            store.set("timeout_done/%s" % sched, b"1")
        else:
            store.get("timeout_done/%s" % sched, timeout_ms=120000)
        torch.cuda.synchronize()  # the kernels that gave up have exited
        alg.close()
    ctx.close()
    if not ok:
        print("MISMATCH rank", rank)
        sys.exit(1)
    print("OK")


def run_custom(store_dir, rank, size):
    """Every custom-function fixture case at P = size (tests/
    test_allreduce_custom.py): gloo::allreduce with a caller's function on
    host buffers, one process per rank, each output against the reference's."""
    import gloo_amd
    from test_allreduce_custom import CASES, buffers, check_result, run_rank
    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(60)
    ctx.connectFullMesh(store)
    bad, n = [], 0
    for c in CASES:
        if c["P"] != size:
            continue
        ins, outs = buffers(c)
        run_rank(ctx, c, ins[rank], outs[rank])
        n += 1
        if not all(check_result(c, o) for o in outs[rank]):
            bad.append(c["name"])
    barrier(store, rank, size, "custom")
    ctx.close()
    print("custom cases %d, wrong %s" % (n, bad[:5]))
    if bad or n == 0:
        print("MISMATCH rank", rank)
        sys.exit(1)
    print("OK")


def run_class_custom(store_dir, rank, size):
    """Every class-custom fixture case at P = size (tests/
    test_allreduce_class_custom.py): AllreduceRingChunked /
    AllreduceHalvingDoubling with a CUSTOM ReductionFunction on host buffers,
    one process per rank, every pointer against the reference's output."""
    import gloo_amd
    from test_allreduce_class_custom import CASES, buffers, check_result, make_alg
    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(60)
    ctx.connectFullMesh(store)
    bad, n = [], 0
    for c in CASES:
        if c["P"] != size:
            continue
        bufs = buffers(c)[rank]
        alg = make_alg(ctx, c, bufs)
        alg.run()
        alg.close()
        n += 1
        if not all(check_result(c, b) for b in bufs):
            bad.append(c["name"])
    barrier(store, rank, size, "class_custom")
    ctx.close()
    print("class custom cases %d, wrong %s" % (n, bad[:5]))
    if bad or n == 0:
        print("MISMATCH rank", rank)
        sys.exit(1)
    print("OK")


def run_dma_abort(store_dir, rank, size):
    """the DMA steps engine enqueues a copy behind the flag
    kernel that waits for its receiver's credit, and HIP runs the copy whatever
    that wait found.  Rank 0 (1 s timeout) gives up on a credit while rank 1
    (30 s) is healthy but late -- its stream is held by a sleep kernel -- so
    rank 0's next copy lands in rank 1's region before rank 1 consumed the
    message there.  Rank 1 must not return that data: the abort mark rank 0
    posted before the copy could start stops rank 1's run, which raises
    IoException naming rank 0 -- long before its own 30 s timeout."""
    import time

    import torch

    import gloo_amd

    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(1 if rank == 0 else 30)
    ctx.connectFullMesh(store)
    n = 1 << 20
    s = torch.cuda.Stream()
    buf = torch.ones(n, device="cuda")
    gloo_amd.set_steps_engine("dma")
    try:
        alg = gloo_amd.AllreduceRingChunked(ctx, [buf], schedule="ring", streams=[s])
    finally:
        gloo_amd.set_steps_engine("auto")
    ok = alg.engine() == "dmasteps"
    torch.cuda.synchronize()
    alg.run()  # a clean run first: every rank holds P everywhere
    s.synchronize()
    ok = ok and bool((buf == size).all().item())
    # cycles of torch.cuda._sleep per second on this GPU
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(1 << 22)
    e1.record()
    e1.synchronize()
    per_s = (1 << 22) / max(1e-6, e0.elapsed_time(e1) / 1e3)
    buf.fill_(1)
    torch.cuda.synchronize()
    barrier(store, rank, size, "armed")
    if rank == 1:
        with torch.cuda.stream(s):
            torch.cuda._sleep(int(per_s * 4))  # rank 1 consumes nothing for ~4 s
    t0 = time.time()
    msg = None
    try:
        alg.run()
        s.synchronize()
        alg.run()  # reports how the run before ended
        s.synchronize()
    except gloo_amd.IoException as e:
        msg = str(e)
    dt = time.time() - t0
    print("rank %d after %.1f s: %s" % (rank, dt, msg), flush=True)
    if rank == 0:
        ok = ok and msg is not None and "Timed out" in msg
    else:
        ok = (ok and msg is not None and "Rank 0 gave up on its DMA steps run" in msg
              and dt < 20)
    barrier(store, rank, size, "reported")
    alg.close()
    ctx.close()
    if not ok:
        print("MISMATCH rank", rank)
        sys.exit(1)
    print("OK")


def run_killpeer(store_dir, rank, size, engine, when):
    """TransportMultiProcTest.IoErrors (gloo/test/transport_test.cc:53-110):
    rank 0 is SIGKILLed; the survivors' next run() must raise IoException
    within 2x the timeout.  engine: host (host-issued ring steps), device
    (the ring's plan kernel), dma (the DMA steps engine), twoshot (the mesh
    kernel).  when: idle (rank 0
    dies while the others are already waiting in run()) or mid (rank 0 dies
    while its own run() is in flight)."""
    import os
    import signal
    import threading
    import time

    import torch

    import gloo_amd

    T = 3.0
    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(T)
    ctx.connectFullMesh(store)
    n = 3 << 20  # 16-byte aligned ring chunks at P = 2, 3, 4 (plan-kernel eligible)
    buf = torch.ones(n, device="cuda")
    if engine == "twoshot":
        alg = gloo_amd.AllreduceRingChunked(ctx, [buf], schedule="mesh")
    else:
        gloo_amd.set_steps_engine(engine)
        alg = gloo_amd.AllreduceRingChunked(ctx, [buf], schedule="ring")
        gloo_amd.set_steps_engine("auto")
    want = {"host": "steps", "device": "devsteps", "dma": "dmasteps",
            "twoshot": "twoshot"}[engine]
    ok = alg.engine() == want
    if not ok:
        print("engine %s, expected %s" % (alg.engine(), want))
    for _ in range(3):
        buf.fill_(1.0)
        torch.cuda.synchronize()
        alg.run()
        ok = ok and bool(torch.all(buf == size).item())
    store.set("warm/%d" % rank, b"1")
    for r in range(size):
        store.get("warm/%d" % r, timeout_ms=60000)
    if rank == 0:
        if when == "mid":
            threading.Timer(0.05, lambda: os.kill(os.getpid(), signal.SIGKILL)).start()
            while True:
                alg.run()
        time.sleep(0.5)
        os.kill(os.getpid(), signal.SIGKILL)
    t0 = time.time()
    try:
        for _ in range(1000):  # 'mid': the peer may finish a few runs first
            alg.run()
        print("NO ERROR after the peer died")
        ok = False
    except gloo_amd.IoException as e:
        dt = time.time() - t0
        print("IoException after %.2f s: %s" % (dt, str(e)[:200]))
        # every engine notices the exit itself, well before the timeout
        ok = ok and dt < T and "Connection closed by peer" in str(e)
    torch.cuda.synchronize()  # kernels that gave up have exited
    alg.close()
    ctx.close()
    if not ok:
        print("MISMATCH rank", rank)
        sys.exit(1)
    print("OK")


def run_churn(store_dir, rank, size):
    """Many algorithms created, run and destroyed back to back on every
    engine (shared blocks come from the context's pool and are reused while
    peers may still be finishing the previous algorithm): every result
    bit-exact, and no file descriptors accumulate (IPC in dmabuf mode passes
    them)."""
    import numpy as np
    import torch

    import gloo_amd
    from helpers import case_inputs
    from oracle import oracle as O

    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(30)
    ctx.connectFullMesh(store)

    def nfd():
        return len(os.listdir("/proc/self/fd"))

    kinds = [("replicated", "auto"), ("mesh", "auto"), ("ring", "device"), ("ring", "host"),
             ("hd", "device"), ("hd", "host"), ("ring", "dma"), ("hd", "dma")]
    sizes = [1000, 4096, 65539, 12345, 1 << 16, 777]
    bad, fds = [], []
    for it in range(36):
        sched, eng = kinds[it % len(kinds)]
        n = sizes[(it // len(kinds)) % len(sizes)]
        ins = case_inputs(size, n, O.FLOAT32, 1, 0, seed=500 + it)
        kind = O.HALVING_DOUBLING if sched == "hd" else O.RING_CHUNKED
        exp = O.allreduce(kind, O.SUM, O.FLOAT32, ins)[rank][0]
        buf = torch.from_numpy(ins[rank][0].copy()).cuda()
        torch.cuda.synchronize()
        gloo_amd.set_steps_engine(eng)
        if sched == "hd":
            alg = gloo_amd.AllreduceHalvingDoubling(ctx, [buf])
        else:
            alg = gloo_amd.AllreduceRingChunked(ctx, [buf], schedule=sched)
        gloo_amd.set_steps_engine("auto")
        for r in range(2):
            buf.copy_(torch.from_numpy(ins[rank][0]))
            torch.cuda.synchronize()
            alg.run()
            got = buf.cpu().numpy()
            if not np.array_equal(got.view(np.uint32), exp.view(np.uint32)):
                bad.append((it, sched, eng, n, alg.engine(), r))
        alg.close()
        fds.append(nfd())
    print("IPC rank %d %s" % (rank, ctx.ipc_stats()), flush=True)
    ctx.close()
    print("fds", fds[:3], "...", fds[-3:])
    if bad:
        print("MISMATCH rank", rank, bad[:10])
        sys.exit(1)
    if fds[-1] > fds[5] + 8:
        print("FD LEAK rank", rank, fds)
        sys.exit(1)
    print("OK")


def run_devsteps(store_dir, rank, size, eng="device"):
    import time

    import numpy as np
    import torch

    import gloo_amd
    from helpers import case_inputs
    from oracle import oracle as O
    from test_reduce_gpu import from_dev, to_dev

    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(20)
    ctx.connectFullMesh(store)
    bad = []

    def same(got, exp):
        return np.array_equal(np.ascontiguousarray(got).view(np.uint8),
                              np.ascontiguousarray(exp).view(np.uint8))

    label = {"device": "devsteps", "dma": "dmasteps"}.get(eng, eng)
    MESH = 100  # the mesh schedule (ring_chunked semantics)

    def make(kind, buf, op=O.SUM, dt=None):
        fn = gloo_amd.ReductionFunction(op)
        if kind == O.HALVING_DOUBLING:
            return gloo_amd.AllreduceHalvingDoubling(ctx, [buf], fn=fn, dtype=dt)
        if kind == O.RING:
            return gloo_amd.AllreduceRing(ctx, [buf], fn=fn, dtype=dt)
        if kind == O.BCUBE:
            return gloo_amd.AllreduceBcube(ctx, [buf], fn=fn, dtype=dt)
        return gloo_amd.AllreduceRingChunked(ctx, [buf], fn=fn, dtype=dt,
                                             schedule="mesh" if kind == MESH else "ring")

    cases = []
    kinds = (O.RING_CHUNKED, O.HALVING_DOUBLING, O.RING, O.BCUBE)
    ctx.base = 3 if size in (3, 9) else 2  # AllreduceBcube's groups
    for kind in kinds:
        for n in (1, 3, 255, 256, 1000, 4099, 65539, 1 << 20, (1 << 22) + 5):
            cases.append((kind, n, O.FLOAT32, O.SUM))
        for dt in (O.FLOAT16, O.BFLOAT16, O.INT32, O.FLOAT64, O.INT8, O.UINT64):
            for op in (O.SUM, O.PRODUCT, O.MAX, O.MIN):
                cases.append((kind, 4099, dt, op))
    gloo_amd.set_steps_engine(eng)
    engines = set()
    for seed, (kind, n, dt, op) in enumerate(cases):
        ins = case_inputs(size, n, dt, 1, 0, seed=200 + seed)
        # the mesh schedule computes ring_chunked's result (same chunks and chains)
        exp = O.allreduce(O.RING_CHUNKED if kind == MESH else kind, op, dt, ins,
                          base=ctx.base)[rank][0]
        buf = to_dev(ins[rank][0], dt)
        alg = make(kind, buf, op, dt)
        # the plan kernel, or host-issued steps where a landing region would
        # be shared across workgroups (glx_plan_sync "safe")
        engines.add(alg.engine())
        print("case %d kind %d n %d dtype %d op %d engine %s" % (seed, kind, n, dt, op,
                                                                 alg.engine()), flush=True)
        if alg.engine() not in (label, "steps"):
            bad.append(("engine", kind, n, alg.engine()))
        for it in range(3):
            buf.copy_(to_dev(ins[rank][0], dt))
            torch.cuda.synchronize()
            alg.run()
            if not same(from_dev(buf, dt), exp):
                bad.append(("class", kind, n, dt, op, it))
        alg.close()
    if label not in engines:
        bad.append(("engine", label, "never ran"))
    n = 65536  # host buffers: staged H2D, kernel, D2H
    ins = case_inputs(size, n, O.FLOAT32, 1, 0, seed=8)
    for kind in (O.RING_CHUNKED, O.HALVING_DOUBLING):
        exp = O.allreduce(kind, O.SUM, O.FLOAT32, ins)[rank][0]
        host = ins[rank][0].copy()
        alg = make(kind, host)
        for it in range(2):
            host[:] = ins[rank][0]
            alg.run()
            if not same(host, exp):
                bad.append(("host", kind, it))
        alg.close()
    A = gloo_amd.AllreduceOptions.Algorithm
    for algo, code in ((A.RING, O.FN_RING), (A.BCUBE, O.FN_BCUBE)):
        for n in (1000, 65536, 1 << 20):
            data = case_inputs(size, n, O.FLOAT32, 1, 0, seed=12)
            exp = O.allreduce_fn(code, O.SUM, O.FLOAT32, [[] for _ in range(size)],
                                 data)[rank][0]
            for it in range(2):
                out = torch.from_numpy(data[rank][0].copy()).cuda()
                torch.cuda.synchronize()
                opts = gloo_amd.AllreduceOptions(ctx)
                opts.setAlgorithm(algo)
                opts.setOutput(out)
                opts.setReduceFunction(gloo_amd.ReductionFunction.sum)
                gloo_amd.allreduce(opts)
                if not same(out.cpu().numpy(), exp):
                    bad.append(("fn", code, n, it))
    # latency: the plan kernel vs the host-issued steps (same bits)
    for kind, label in ((O.RING_CHUNKED, "ring"), (O.HALVING_DOUBLING, "hd")):
        for n in (1024, 65536, 1 << 20, 3 << 22):
            for e in (eng, "host"):
                gloo_amd.set_steps_engine(e)
                buf = torch.zeros(n, device="cuda")
                torch.cuda.synchronize()
                alg = make(kind, buf)
                for _ in range(3):
                    alg.run()
                iters = 20 if n <= (1 << 20) else 5
                t0 = time.perf_counter()
                for _ in range(iters):
                    alg.run()
                us = (time.perf_counter() - t0) / iters * 1e6
                print("LAT rank %d P %d %s elems %d engine %s us %.1f"
                      % (rank, size, label, n, alg.engine(), us), flush=True)
                alg.close()
    if eng == "dma":
        gloo_amd.set_steps_engine("dma")
        # with a caller's stream run() only enqueues: K runs back to back on
        # one buffer, one wait at the end; each run reduces the previous
        # run's result (int32 sums wrap alike on every rank and in the oracle)
        s = torch.cuda.Stream()
        n, K = 65539, 5
        ins = case_inputs(size, n, O.INT32, 1, 0, seed=41)
        exp = ins[rank][0]
        cur = ins
        for _ in range(K):
            exp = O.allreduce(O.RING_CHUNKED, O.SUM, O.INT32, cur)[rank][0]
            cur = [[exp.copy()] for _ in range(size)]
        buf = to_dev(ins[rank][0], O.INT32)
        torch.cuda.synchronize()
        alg = gloo_amd.AllreduceRingChunked(ctx, [buf], streams=[s], dtype=O.INT32,
                                            schedule="ring")
        for _ in range(K):
            alg.run()
        s.synchronize()
        if alg.engine() != "dmasteps" or not same(from_dev(buf, O.INT32), exp):
            bad.append(("async stream runs", alg.engine()))
        # a captured run would replay host-counted message numbers: refused
        graph = torch.cuda.CUDAGraph()
        refused = ""
        try:
            with torch.cuda.graph(graph, stream=s):
                alg.run()
        except gloo_amd.EnforceNotMet as e:
            refused = str(e)
        except RuntimeError as e:  # the capture's end after the refusal
            refused = refused or str(e)
        if "HIP graph" not in refused:
            bad.append(("capture not refused", refused[:120]))
        s.synchronize()
        alg.close()
    gloo_amd.set_steps_engine("auto")
    gloo_amd.set_mesh_engine("device")
    store.set("done/%d" % rank, b"1")
    for r in range(size):
        store.get("done/%d" % r, timeout_ms=60000)
    print("IPC rank %d %s" % (rank, ctx.ipc_stats()), flush=True)
    ctx.close()
    if bad:
        print("MISMATCH rank", rank, bad[:10])
        sys.exit(1)
    print("OK")


def run_device(store_dir, rank, size, mode):
    import time

    import numpy as np
    import torch

    import gloo_amd
    from helpers import case_inputs
    from oracle import oracle as O

    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(20)
    ctx.connectFullMesh(store)
    bad = []

    def same(got, exp):
        return np.array_equal(np.ascontiguousarray(got).view(np.uint8),
                              np.ascontiguousarray(exp).view(np.uint8))

    from test_reduce_gpu import from_dev, to_dev

    sched = "replicated" if mode == "oneshot" else "mesh"
    cases = []
    sizes = [1, 3, 255, 256, 1024, 4099, 65539, 262144, 1 << 20]
    if mode == "twoshot":
        sizes += [(1 << 22) + 5, 3 << 22]
    for n in sizes:
        cases.append((n, O.FLOAT32, O.SUM))
    for dt in (O.FLOAT16, O.BFLOAT16, O.INT32, O.FLOAT64, O.INT8, O.UINT64):
        for op in (O.SUM, O.PRODUCT, O.MAX, O.MIN):
            cases.append((4099, dt, op))
    cases.append((77777, O.FLOAT16, O.SUM))
    for seed, (n, dt, op) in enumerate(cases):
        ins = case_inputs(size, n, dt, 1, 0, seed=100 + seed)
        exp = O.allreduce(O.RING_CHUNKED, op, dt, ins)[rank][0]
        buf = to_dev(ins[rank][0], dt)
        alg = gloo_amd.AllreduceRingChunked(ctx, [buf], fn=gloo_amd.ReductionFunction(op),
                                           schedule=sched, dtype=dt)
        if alg.engine() != mode:
            bad.append(("engine", n, dt, op, alg.engine()))
        for it in range(3):
            buf.copy_(to_dev(ins[rank][0], dt))
            torch.cuda.synchronize()
            alg.run()
            got = from_dev(buf, dt)
            if not same(got, exp):
                bad.append(("class", n, dt, op, it))
        alg.close()
    # host buffers (numpy): staged H2D, kernel, D2H
    n = 4099
    ins = case_inputs(size, n, O.FLOAT32, 1, 0, seed=7)
    exp = O.allreduce(O.RING_CHUNKED, O.SUM, O.FLOAT32, ins)[rank][0]
    host = ins[rank][0].copy()
    alg = gloo_amd.AllreduceRingChunked(ctx, [host], schedule=sched)
    for it in range(2):
        host[:] = ins[rank][0]
        alg.run()
        if not same(host, exp):
            bad.append(("host", n, it))
    alg.close()
    # function style: RING's result, one round (UNSPECIFIED at a small size)
    # or over all links (RING_MESH)
    fn_algo = (gloo_amd.AllreduceOptions.Algorithm.UNSPECIFIED if mode == "oneshot"
               else gloo_amd.AllreduceOptions.Algorithm.RING_MESH)
    for n in (1000, 65536, 1 << 20):
        data = case_inputs(size, n, O.FLOAT32, 1, 0, seed=11)
        exp = O.allreduce_fn(O.FN_RING, O.SUM, O.FLOAT32, [[] for _ in range(size)],
                             data)[rank][0]
        for it in range(2):
            out = torch.from_numpy(data[rank][0].copy()).cuda()
            opts = gloo_amd.AllreduceOptions(ctx)
            opts.setAlgorithm(fn_algo)
            opts.setOutput(out)
            opts.setReduceFunction(gloo_amd.ReductionFunction.sum)
            gloo_amd.allreduce(opts)
            if not same(out.cpu().numpy(), exp):
                bad.append(("fn", n, it))
    # latency of the device-driven engine vs the host-issued steps (same bits)
    lat_sizes = (1024, 65536, 262144) if mode == "oneshot" else (65536, 1 << 20, 1 << 24)
    for n in lat_sizes:
        for eng in ("device", "steps"):
            if mode == "twoshot":
                gloo_amd.set_mesh_engine(eng)
            elif eng == "steps":
                continue
            buf = torch.zeros(n, device="cuda")
            alg = gloo_amd.AllreduceRingChunked(ctx, [buf], schedule=sched)
            for _ in range(5):
                alg.run()
            iters = 50 if n <= (1 << 20) else 10
            t0 = time.perf_counter()
            for _ in range(iters):
                alg.run()
            us = (time.perf_counter() - t0) / iters * 1e6
            print("LAT rank %d P %d elems %d engine %s us %.1f" % (rank, size, n, alg.engine(),
                                                                    us))
            alg.close()
    gloo_amd.set_mesh_engine("device")
    store.set("done/%d" % rank, b"1")
    for r in range(size):
        store.get("done/%d" % r, timeout_ms=60000)
    print("IPC rank %d %s" % (rank, ctx.ipc_stats()), flush=True)
    ctx.close()
    if bad:
        print("MISMATCH rank", rank, bad[:10])
        sys.exit(1)
    print("OK")


def run_big(store_dir, rank, size, policy):
    import torch

    import gloo_amd
    assert size == 2, "big: P = 2 (the result is x0 + x1 exactly)"
    n = (1 << 29) + 4096 + 5  # fp32: 2 GiB + 16 KiB + 20 B per rank, odd tail
    dev = torch.device("cuda", 0)

    def inp(r):
        g = torch.Generator(device=dev).manual_seed(777 + r)
        return torch.rand(n, device=dev, generator=g) * 2 - 1
    buf = inp(rank)
    torch.cuda.synchronize()
    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(120)
    ctx.connectFullMesh(store)
    gloo_amd.set_steps_engine("device")
    gloo_amd.set_engine_streams(policy)
    try:
        alg = gloo_amd.AllreduceRingChunked(ctx, [buf], schedule="ring")
    finally:
        gloo_amd.set_steps_engine("auto")
        gloo_amd.set_engine_streams("auto")
    print("big rank %d engine %s fast %s" % (rank, alg.engine(), alg.fast_streams()), flush=True)
    bad = []
    if alg.engine() != "devsteps" or alg.fast_streams() != (policy == "fast"):
        bad.append(("engine", alg.engine(), alg.fast_streams()))
    for it in range(2):
        if it:
            buf.copy_(inp(rank))
            torch.cuda.synchronize()
        alg.run()
        exp = inp(0) + inp(1)
        diff = int((buf.view(torch.int32) != exp.view(torch.int32)).sum().item())
        if diff:
            first = int((buf.view(torch.int32) != exp.view(torch.int32)).nonzero()[0].item())
            bad.append(("run", it, diff, first))
        del exp
        torch.cuda.empty_cache()
    alg.close()
    store.set("done/%d" % rank, b"1")
    for r in range(size):
        store.get("done/%d" % r, timeout_ms=120000)
    ctx.close()
    if bad:
        print("MISMATCH rank", rank, bad[:10])
        sys.exit(1)
    print("OK")


def run_maxcount(store_dir, rank, size):
    """count = INT_MAX (2^31 - 1, odd), the largest the reference's class
    constructors take (gloo/allreduce_ring_chunked.h:25,
    allreduce_halving_doubling.h:70): int8 (2 GiB - 1 B per rank) and float16
    (4 GiB - 2 B: element offsets times the element size pass 2^32) through
    the ring on the plan kernel, the host-issued steps and the DMA steps
    engine, the mesh and halving-doubling on the plan kernel.  P = 2: the
    sum commutes, so the result is x0 + x1 bit for bit (int8 wraps; float16
    adds in fp32 and rounds once, as torch does).  Every case runs: messages
    above 512 MiB go as pieces in regions of their own (plan.h
    splitMessages), so no landing block another process imports reaches the
    2 GiB at which the IPC import hangs (Context::kIpcMaxBlockBytes)."""
    import time

    import torch

    import gloo_amd
    assert size == 2, "maxcount: P = 2 (the result is x0 + x1 exactly)"
    # diagnostics: MAXCOUNT_N / _SCHED / _DTYPE / _TIMEOUT narrow the run
    n = int(os.environ.get("MAXCOUNT_N", (1 << 31) - 1))
    only = os.environ.get("MAXCOUNT_SCHED", "").split(",")
    dts = os.environ.get("MAXCOUNT_DTYPE", "int8,float16").split(",")
    dev = torch.device("cuda", 0)

    def inp(r, dt):
        g = torch.Generator(device=dev).manual_seed(4242 + r)
        if dt == torch.int8:
            return torch.randint(-128, 128, (n,), dtype=dt, device=dev, generator=g)
        return torch.rand(n, dtype=dt, device=dev, generator=g) * 2 - 1
    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(int(os.environ.get("MAXCOUNT_TIMEOUT", 120)))
    ctx.connectFullMesh(store)
    bad = []
    # (steps engine, schedule, engine it must get or "refused") per dtype:
    # the mesh lands a whole range per peer slot array (4 arrays of P x ~S/P);
    # float16's halving-doubling receives half its 4 GiB buffer in one region;
    # the automatic schedule takes the ring at these sizes (plan.h
    # kMeshMaxBytes), on the host-issued steps (ranks share the GPU, > 32 MiB)
    # round 6: messages above 512 MiB go as pieces, each in a
    # region of its own (plan.h splitMessages), so nothing is refused: the
    # mesh (whose two-shot kernel would need ~S per slot array) runs as
    # host-issued steps; float16's ring and both halving-doublings split
    cases = {
        torch.int8: (("device", "ring", "devsteps"), ("host", "ring", "steps"),
                     ("dma", "ring", "dmasteps"), ("auto", "mesh", "steps"),
                     ("device", "hd", "devsteps"), ("auto", "auto", "steps")),
        torch.float16: (("device", "ring", "devsteps"), ("host", "ring", "steps"),
                        ("dma", "ring", "dmasteps"), ("auto", "mesh", "steps"),
                        ("device", "hd", "devsteps"), ("dma", "hd", "dmasteps"),
                        ("auto", "auto", "steps")),
    }
    for dt, bits in ((torch.int8, torch.int8), (torch.float16, torch.int16)):
        if str(dt).split(".")[1] not in dts:
            continue
        exp = inp(0, dt) + inp(1, dt)
        buf = inp(rank, dt)
        for eng, sched, want in cases[dt]:
            if only != [""] and sched not in only:
                continue
            gloo_amd.set_steps_engine(eng)
            try:
                if sched == "hd":
                    alg = gloo_amd.AllreduceHalvingDoubling(ctx, [buf])
                else:
                    alg = gloo_amd.AllreduceRingChunked(ctx, [buf], schedule=sched)
            except gloo_amd.EnforceNotMet as e:
                alg = None
                msg = str(e)
            finally:
                gloo_amd.set_steps_engine("auto")
            if alg is None:
                ok = want == "refused" and "IPC imports of 2 GiB" in msg
                print("maxcount rank %d %s %s refused (%s): %s" % (
                    rank, dt, sched, "expected" if ok else "UNEXPECTED", msg[:160]), flush=True)
                if not ok:
                    bad.append(("refused", str(dt), sched, msg[:200]))
                continue
            if want == "refused" or alg.count != n or alg.engine() != want:
                bad.append(("engine", str(dt), sched, alg.count, alg.engine(), want))
            buf.copy_(inp(rank, dt))
            torch.cuda.synchronize()
            print("maxcount rank %d %s %s engine %s: run" % (rank, dt, sched, alg.engine()),
                  flush=True)
            t0 = time.perf_counter()
            alg.run()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            diff = int((buf.view(bits) != exp.view(bits)).sum().item())
            if diff:
                first = int((buf.view(bits) != exp.view(bits)).nonzero()[0].item())
                bad.append(("run", str(dt), sched, alg.engine(), diff, first))
            print("maxcount rank %d %s %s engine %s %.1f ms %s" % (
                rank, dt, sched, alg.engine(), ms, "ok" if not diff else "MISMATCH %d" % diff),
                flush=True)
            alg.close()
        del exp, buf
        torch.cuda.empty_cache()
    store.set("done/%d" % rank, b"1")
    for r in range(size):
        store.get("done/%d" % r, timeout_ms=120000)
    ctx.close()
    if bad:
        print("MISMATCH rank", rank, bad[:10])
        sys.exit(1)
    print("OK")


def run_linkprobe(store_dir, rank, size):
    import torch

    import gloo_amd
    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(60)
    ctx.connectFullMesh(store)
    bad = []
    for k in range(size):
        if k == rank:
            continue
        info = ctx.peer_info(k)
        # one GPU: every peer is on this rank's own GPU, nothing asked of a link
        if not (info["same_gpu"] and info["device"] == 0 and info["can_access_peer"] is None
                and info["native_atomics"] is None):
            bad.append(("peer_info", k, info))
    nbytes = (8 << 20) + 4096
    probe = gloo_amd.rendezvous.LinkProbe(ctx, nbytes)
    for pattern, name in ((probe.RING, "ring"), (probe.MESH, "mesh")):
        for engine in (probe.DMA, probe.KERNEL):
            barrier(store, rank, size, "lp%s%d" % (name, engine))
            secs, link = probe.run(pattern, engine, 128, 3)
            want = nbytes  # both patterns: nbytes on every link they use
            if not (secs > 0 and link == want):
                bad.append(("probe", name, engine, secs, link, want))
            print("LINK rank %d %s engine %d %.1f GB/s" % (rank, name, engine,
                                                         link * 3 / secs / 1e9), flush=True)
    barrier(store, rank, size, "lpdone")
    probe.close()
    # the context goes on working after the probe: its blocks went back to the pool
    buf = torch.full((1 << 20,), float(rank + 1), device="cuda")
    alg = gloo_amd.AllreduceRingChunked(ctx, [buf])
    alg.run()
    if not bool((buf == size * (size + 1) / 2).all().item()):
        bad.append(("allreduce after probe",))
    alg.close()
    barrier(store, rank, size, "end")
    ctx.close()
    if bad:
        print("MISMATCH rank", rank, bad[:10])
        sys.exit(1)
    print("OK")


def run_engine_choice(store_dir, rank, size):
    """The engine the automatic policy gives the ring on a shared GPU under
    this process's GPU_MAX_HW_QUEUES (HipPlanExecutor::deviceEnginesAvailable:
    processes sharing a GPU get the device engines only within the
    hardware-queue budget), and one exact run of it."""
    import torch

    import gloo_amd
    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(60)
    ctx.connectFullMesh(store)
    buf = torch.full((4099,), float(rank + 1), device="cuda")
    alg = gloo_amd.AllreduceRingChunked(ctx, [buf], schedule="ring")
    alg.run()
    torch.cuda.synchronize()
    ok = bool((buf == size * (size + 1) / 2).all().item())
    print("ENGINE rank %d %s" % (rank, alg.engine()), flush=True)
    alg.close()
    store.set("done/%d" % rank, b"1")
    for r in range(size):
        store.get("done/%d" % r, timeout_ms=60000)
    ctx.close()
    if not ok:
        print("MISMATCH rank", rank)
        sys.exit(1)
    print("OK")


def run_graph(store_dir, rank, size, replays):
    """HIP graph capture of run() on every device engine: each algorithm (ring
    and halving-doubling on the plan kernel, the mesh on the two-shot kernel,
    the replicated schedule on the one-shot kernel, on a caller's stream)
    runs once eagerly, is captured into a graph with torch.cuda.graph, and
    then the graph is replayed with fresh inputs, mixed with eager runs --
    the kernels take their run count / epoch from the device (kernels.h
    runCtr, epochCtr), so replays and eager runs interleave in one sequence
    on every rank.  Exact sums of integer-valued inputs as in the soak."""
    import torch

    import gloo_amd

    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(30)
    ctx.connectFullMesh(store)
    n = 1 << 20
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream()

    def inputs(r, it):
        g = torch.Generator(device=dev)
        g.manual_seed(7919 * it + r)
        return torch.randint(-64, 64, (n,), generator=g, device=dev, dtype=torch.int32)

    bad, engines = [], {}
    for kind in ("ring", "hd", "mesh", "repl"):
        buf = torch.empty(n, dtype=torch.float32, device=dev)
        if kind == "hd":
            alg = gloo_amd.AllreduceHalvingDoubling(ctx, [buf], streams=[s])
        else:
            sched = {"ring": "ring", "mesh": "mesh", "repl": "replicated"}[kind]
            alg = gloo_amd.AllreduceRingChunked(ctx, [buf], streams=[s], schedule=sched)
        engines[kind] = alg.engine()

        def check(it):
            s.synchronize()
            expect = sum(inputs(r, it).to(torch.int64) for r in range(size))
            got = buf.to(torch.int64)
            if not torch.equal(got, expect):
                bad.append((kind, it, int((got != expect).sum())))

        with torch.cuda.stream(s):
            buf.copy_(inputs(rank, 0).to(torch.float32))
        alg.run()  # eager: resolves the peers, builds the step table
        check(0)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            buf.copy_(inputs(rank, 1).to(torch.float32))
        s.synchronize()
        with torch.cuda.graph(graph, stream=s):
            alg.run()
        # capturing launched nothing: the graph's first replay is run 1
        with torch.cuda.stream(s):
            graph.replay()
        check(1)
        for it in range(2, replays + 2):
            with torch.cuda.stream(s):
                buf.copy_(inputs(rank, it).to(torch.float32))
                if it % 4 == 0:
                    alg.run()       # eager runs between replays share the count
                else:
                    graph.replay()
            check(it)
        s.synchronize()
        # run() on its fixed stream records no done event per call (each
        # would cost the stream microseconds: DESIGN 5b, small messages)
        if alg.transport_stats()["done_events"] != 0:
            bad.append((kind, "done_events", alg.transport_stats()["done_events"]))
        del graph
        alg.close()
    store.set("graph/done/%d" % rank, b"1")
    for r in range(size):
        store.get("graph/done/%d" % r, timeout_ms=60000)
    print("ENGINES rank %d %s" % (rank, engines))
    if bad:
        print("MISMATCH rank %d %s" % (rank, bad[:10]))
        sys.exit(1)
    print("OK")


def run_graph_overlap(store_dir, rank, size, kind, close_first=False):
    """launches of one algorithm must not overlap -- a
    graph captured on the algorithm's stream but replayed on another stream
    while an eager run is still in flight would take the same run number /
    epoch and share landing slots.  The kernels now detect it
    (xgmi_kernels.hip launch_number): rank 0 starts an eager run that waits
    for rank 1 (which starts its own 0.5 s later) and replays the captured
    run on a second stream meanwhile; one of the two launches must report
    the overlap, and rank 0's next call raises EnforceNotMet naming it.
    Rank 1's run then either completes or times out (IoException) within
    the context's 5 s timeout; nothing hangs.

    close_first: rank 0 frees the algorithm right after the overlap instead
    of calling it again, and rank 1 never starts its run; the free must not
    wait out the (20 s) timeout for launches that stopped early
    (HipPlanExecutor::deviceReported)."""
    import time

    import torch

    import gloo_amd
    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(20 if close_first else 5)
    ctx.connectFullMesh(store)
    n = 1 << 16
    dev = torch.device("cuda:0")
    # s2 at another priority: a hardware queue of its own, so the replay can
    # run beside the eager launch instead of queueing behind it
    s, s2 = torch.cuda.Stream(), torch.cuda.Stream(priority=-1)
    buf = torch.full((n,), float(rank + 1), device=dev)
    sched = {"ring": "ring", "mesh": "mesh", "repl": "replicated"}[kind]
    alg = gloo_amd.AllreduceRingChunked(ctx, [buf], streams=[s], schedule=sched)
    engine = alg.engine()
    torch.cuda.synchronize()
    alg.run()  # eager run 0 on every rank: resolves the peers
    s.synchronize()
    ok0 = bool((buf == size * (size + 1) / 2).all().item())
    verdict = "none"
    if rank == 0:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            alg.run()
        store.set("overlap/go", b"1")
        alg.run()  # eager run 1 on s: waits for rank 1
        with torch.cuda.stream(s2):
            graph.replay()  # NOT ordered after the eager run
        s.synchronize()
        s2.synchronize()
        if close_first:
            t0 = time.time()
            alg.close()
            took = time.time() - t0
            verdict = "closed in %.2f s" % took
            print("VERDICT rank 0 %s engine %s first %s" % (verdict, engine, ok0), flush=True)
            store.set("overlap/done/0", b"1")
            store.get("overlap/done/1", timeout_ms=60000)
            if not ok0 or took > 3.0:
                sys.exit(1)
            print("OK")
            return
        try:
            alg.run()
            s.synchronize()
            alg.run()
            s.synchronize()
            verdict = "no error"
        except gloo_amd.EnforceNotMet as e:
            verdict = "overlap" if "still running" in str(e) else "enforce: " + str(e)[:200]
        except gloo_amd.IoException as e:
            verdict = "io: " + str(e)[:200]
        del graph
    elif close_first:
        store.get("overlap/done/0", timeout_ms=60000)
        verdict = "idle"
    else:
        store.get("overlap/go", timeout_ms=60000)
        time.sleep(0.5)
        try:
            alg.run()
            s.synchronize()
            verdict = "completed"
        except gloo_amd.IoException:
            verdict = "timed out"
    print("VERDICT rank %d %s engine %s first %s" % (rank, verdict, engine, ok0), flush=True)
    try:
        alg.close()
    except gloo_amd.Exception:
        pass
    store.set("overlap/done/%d" % rank, b"1")
    for r in range(size):
        store.get("overlap/done/%d" % r, timeout_ms=60000)
    if not ok0 or (rank == 0 and verdict != "overlap"):
        sys.exit(1)
    print("OK")


def run_soak(store_dir, rank, size, runs, uneven="", n=1 << 20):
    """One instance of each device engine's algorithm run `runs` times back to
    back (a training job's shape: the run counter, the message numbers
    j * perRun + seq and the landing slots alternate across many kernel
    boundaries), fresh inputs every run: small integers in fp32, generated on
    the device from a (rank, run) seed by every rank for every rank, so the
    exact sum is each rank's own check -- any order gives the same bits, and
    a stale slot, a lost flag or a message landing in the wrong run shows up
    as a wrong element.

    uneven: the guide's hand-off test condition (MI355X_MICROARCH.md, "Test
    every hand-off under UNEVEN load"): "delays" -- every rank starts each
    run after a random delay of up to 2 ms, so workgroups arrive at their
    flags at different times; "uneven" -- also a GEMM stream busy on rank 0's
    GPU beside the collective, so some CUs are taken.  On the device engines
    (the rehearsal's opt-in, GLOO_AMD_DEVICE_ENGINES=shared) this needs two
    hardware queues per process: with one (8 ranks sharing the GPU) the GEMM
    sits ahead of the collective in rank 0's only queue while the other
    ranks' collectives hold the CUs waiting for rank 0 -- a cycle that exists
    only when ranks share a GPU, which is why the automatic choice keeps such
    ranks on host-issued steps.

    n: elements per rank.  A small n (a few thousand) makes every
    workgroup's share of a landing slot a few hundred bytes that its CU read
    two runs before (the slots alternate): L1-warm re-reads, the guide's
    near-certain stale case without an acquire (MI355X_MICROARCH.md,
    "Stale without an agent-scope acquire") -- the sharp detector for the
    test-only broken sync modes (tests/test_sync_control_gpu.py)."""
    import random
    import time

    import torch

    import gloo_amd

    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(30)
    ctx.connectFullMesh(store)
    # 2^20 (default): a length the plan kernel takes at every P here (ragged
    # lengths whose chunks land at different 16-byte phases in one region keep
    # the host-issued steps, plan.h SyncTable::safe; the fuzz covers those)
    dev = torch.device("cuda:0")

    def inputs(r, it):
        g = torch.Generator(device=dev)
        g.manual_seed(1000003 * it + r)
        return torch.randint(-64, 64, (n,), generator=g, device=dev, dtype=torch.int32)

    # above 32 MiB per rank the automatic choice for processes sharing a GPU
    # runs the ring on host-issued steps (executor_device.cc kDevStepsMaxBytes):
    # "ring_dev" keeps the plan kernel there too (the north star's engine at
    # its own size, e.g. the release-side control at 2^26)
    big = n * 4 > (32 << 20)
    keys = ("ring", "hd", "mesh", "repl", "ring_host", "ring_dma", "hd_dma") + (
        ("ring_dev",) if big else ())
    bufs = {k: torch.empty(n, dtype=torch.float32, device=dev) for k in keys}
    algs = {
        "ring": gloo_amd.AllreduceRingChunked(ctx, [bufs["ring"]], schedule="ring"),
        "hd": gloo_amd.AllreduceHalvingDoubling(ctx, [bufs["hd"]]),
        "mesh": gloo_amd.AllreduceRingChunked(ctx, [bufs["mesh"]], schedule="mesh"),
        "repl": gloo_amd.AllreduceRingChunked(ctx, [bufs["repl"]], schedule="replicated"),
    }
    # and the host-issued steps (shm delivery / credit counters across runs)
    gloo_amd.set_steps_engine("host")
    try:
        algs["ring_host"] = gloo_amd.AllreduceRingChunked(ctx, [bufs["ring_host"]],
                                                          schedule="ring")
    finally:
        gloo_amd.set_steps_engine("auto")
    # and the DMA steps engine (flag words counting across runs; allowed for
    # processes sharing a GPU in every mode but "off": its waits hold one wave)
    gloo_amd.set_steps_engine("dma")
    try:
        algs["ring_dma"] = gloo_amd.AllreduceRingChunked(ctx, [bufs["ring_dma"]],
                                                         schedule="ring")
        algs["hd_dma"] = gloo_amd.AllreduceHalvingDoubling(ctx, [bufs["hd_dma"]])
    finally:
        gloo_amd.set_steps_engine("auto")
    if big:
        gloo_amd.set_steps_engine("device")
        try:
            algs["ring_dev"] = gloo_amd.AllreduceRingChunked(ctx, [bufs["ring_dev"]],
                                                             schedule="ring")
        finally:
            gloo_amd.set_steps_engine("auto")
    engines = {k: a.engine() for k, a in algs.items()}
    rng = random.Random(rank)
    side = torch.cuda.Stream() if uneven == "uneven" and rank == 0 else None
    if side is not None:
        x = torch.randn(2048, 2048, device=dev)
    bad = []
    for it in range(runs):
        mine = inputs(rank, it).to(torch.float32)
        expect = sum(inputs(r, it).to(torch.int64) for r in range(size))
        for k, a in algs.items():
            bufs[k].copy_(mine)
            torch.cuda.synchronize()
            if uneven:
                if side is not None:
                    with torch.cuda.stream(side):
                        for _ in range(4):
                            x = torch.tanh(x @ x)  # busy CUs while the collective runs
                time.sleep(rng.random() * 2e-3)
            a.run()
            got = bufs[k].to(torch.int64)
            if not torch.equal(got, expect):
                bad.append((k, it, int((got != expect).sum())))
        if it % 50 == 0:
            print("SOAK rank %d run %d ok so far: %s" % (rank, it, not bad), flush=True)
    if side is not None:
        side.synchronize()
    for a in algs.values():
        a.close()
    store.set("soak/done/%d" % rank, b"1")
    for r in range(size):
        store.get("soak/done/%d" % r, timeout_ms=60000)
    print("ENGINES rank %d %s" % (rank, engines))
    counts = {}
    for k, _, _ in bad:
        counts[k] = counts.get(k, 0) + 1
    print("BADRUNS rank %d %s of %d runs each" % (rank, counts, runs), flush=True)
    if bad:
        print("MISMATCH rank %d %s" % (rank, bad[:10]))
        sys.exit(1)
    print("OK")


def run_fuzz(store_dir, rank, size, seed):
    """Randomized cases on the device engines, one process per rank: every
    rank draws the same sequence (a shared seed) of (class or function-style
    algorithm, schedule, length, dtype, op, host or device buffer, runs, and
    -- for the step schedules -- the DMA steps engine in about a third of the
    cases) and compares its own output with the oracle bit for bit.  The grid tests fix
    their sizes; this walks lengths and combinations off them."""
    import random

    import numpy as np
    import torch

    import gloo_amd
    from helpers import case_inputs
    from oracle import oracle as O
    from test_reduce_gpu import from_dev, to_dev

    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(30)
    ctx.connectFullMesh(store)
    rng = random.Random(seed)
    dtypes = [O.FLOAT32, O.FLOAT16, O.BFLOAT16, O.INT32, O.INT64, O.FLOAT64, O.INT8, O.UINT64]
    ops = [O.SUM, O.PRODUCT, O.MAX, O.MIN]
    kinds = ["ring_chunked", "halving_doubling", "mesh", "replicated", "ring", "bcube",
             "fn_ring", "fn_bcube"]
    bad = []
    engines = {}
    ncases = int(os.environ.get("FUZZ_CASES", "100"))
    # a second stream of draws (so the cases above stay the seed's): whether
    # the step schedules run on the DMA steps engine this case
    erng = random.Random(seed * 7919 + 1)
    for case in range(ncases):
        kind = rng.choice(kinds)
        dma = erng.random() < 0.35 and kind not in ("mesh", "replicated")
        n = rng.choice([rng.randint(1, 64), rng.randint(65, 70000), rng.randint(70001, 1 << 21)])
        dt = rng.choice(dtypes)
        op = rng.choice(ops) if dt not in (O.FLOAT32,) else rng.choice([O.SUM, O.SUM, O.MAX])
        host = rng.random() < 0.15 and dt not in (O.FLOAT16, O.BFLOAT16)
        runs = rng.choice([1, 2])
        base = rng.choice([2, 3]) if kind == "bcube" else 2
        ins = case_inputs(size, n, dt, 1, 0, seed=1000 + case)
        if kind.startswith("fn_"):
            code = O.FN_BCUBE if kind == "fn_bcube" else O.FN_RING
            exp = O.allreduce_fn(code, op, dt, [[] for _ in range(size)], ins)[rank][0]
        else:
            code = {"ring_chunked": O.RING_CHUNKED, "halving_doubling": O.HALVING_DOUBLING,
                    "mesh": O.RING_CHUNKED, "replicated": O.RING_CHUNKED, "ring": O.RING,
                    "bcube": O.BCUBE}[kind]
            exp = O.allreduce(code, op, dt, ins, base=base)[rank][0]
        ctx.base = base
        fn = gloo_amd.ReductionFunction(op)
        gloo_amd.set_steps_engine("dma" if dma else "auto")
        for it in range(runs):
            buf = ins[rank][0].copy() if host else to_dev(ins[rank][0], dt)
            torch.cuda.synchronize()
            if kind.startswith("fn_"):
                A = gloo_amd.AllreduceOptions.Algorithm
                opts = gloo_amd.AllreduceOptions(ctx)
                opts.setAlgorithm(A.BCUBE if kind == "fn_bcube" else A.RING)
                opts.setOutputs([buf], dtype=dt)
                opts.setReduceFunction(fn)
                gloo_amd.allreduce(opts)
                eng = "fn"
            else:
                dtype_arg = dt  # explicit: uint64 data lives in an int64 tensor
                if kind == "halving_doubling":
                    alg = gloo_amd.AllreduceHalvingDoubling(ctx, [buf], fn=fn, dtype=dtype_arg)
                elif kind == "ring":
                    alg = gloo_amd.AllreduceRing(ctx, [buf], fn=fn, dtype=dtype_arg)
                elif kind == "bcube":
                    alg = gloo_amd.AllreduceBcube(ctx, [buf], fn=fn, dtype=dtype_arg)
                else:
                    sched = {"ring_chunked": "ring", "mesh": "mesh",
                             "replicated": "replicated"}[kind]
                    alg = gloo_amd.AllreduceRingChunked(ctx, [buf], fn=fn, dtype=dtype_arg,
                                                        schedule=sched)
                eng = alg.engine()
                alg.run()
                alg.close()
            got = buf if host else from_dev(buf, dt)
            ok = np.array_equal(np.ascontiguousarray(got).view(np.uint8),
                                np.ascontiguousarray(exp).view(np.uint8))
            engines[eng] = engines.get(eng, 0) + 1
            if not ok:
                bad.append((case, kind, n, dt, op, host, base, eng, it))
        gloo_amd.set_steps_engine("auto")
        print("FUZZ rank %d case %d %s n %d dtype %d op %d host %s base %d engine %s %s"
              % (rank, case, kind, n, dt, op, host, base, eng,
                 "MISMATCH" if bad and bad[-1][0] == case else "ok"), flush=True)
    store.set("done/%d" % rank, b"1")
    for r in range(size):
        store.get("done/%d" % r, timeout_ms=120000)
    print("ENGINES rank %d %s" % (rank, engines), flush=True)
    ctx.close()
    if bad:
        print("MISMATCH rank", rank, bad[:10])
        sys.exit(1)
    print("OK")


def barrier(store, rank, size, tag):
    store.set("bar/%s/%d" % (tag, rank), b"1")
    for r in range(size):
        store.get("bar/%s/%d" % (tag, r), timeout_ms=60000)


def run_scale(store_dir, rank, size, group):
    """BASELINE.json configs at their full size against the reference's own
    output digests (tests/golden/scale_golden.json, made by make_golden.py
    scale): cfg3 ring_chunked fp32 1K..16M elements, cfg4 halving_doubling
    256 MiB, cfg5 ring_chunked fp16 (and bf16, oracle-pinned only) 1 GiB, on
    every engine the product has for the schedule.  Inputs are regenerated
    here with the generator's seed; their digests are checked too."""
    import hashlib
    import json
    import time

    import numpy as np
    import torch

    import gloo_amd
    from oracle import oracle as O
    from test_reduce_gpu import from_dev, to_dev

    if group == "ns":
        # the north-star size (2^26 fp32 = 256 MiB per rank) at this P, ring and
        # halving-doubling: the digests bench.py's N > 1 line checks
        # (tests/golden/bench_golden.json, make_golden.py bench)
        with open(os.path.join(HERE, "golden", "bench_golden.json")) as f:
            cases = [c for c in json.load(f)["cases"] if c["P"] == size]
    else:
        with open(os.path.join(HERE, "golden", "scale_golden.json")) as f:
            cases = json.load(f)["cases"]
        if group == "cfg34":
            cases = [c for c in cases if c["dtype"] == O.FLOAT32]
        else:
            cases = [c for c in cases if c["dtype"] != O.FLOAT32]
    assert cases and all(c["P"] == size for c in cases), "scale cases are for P=%d" % size

    def sha(a):
        h = hashlib.sha256()
        h.update(np.ascontiguousarray(a).view(np.uint8).tobytes())
        return h.hexdigest()

    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(120)
    ctx.connectFullMesh(store)
    bad = []
    for c in cases:
        N, dt = c["N"], c["dtype"]
        x = O.fill(dt, N, 0, seed=c["seed"], rank=rank)
        if sha(x) != c["input_sha256"][rank]:
            bad.append(("input", c["name"]))
            continue
        ring = c["algo"] == O.RING_CHUNKED
        engines = [("device", "ring"), ("host", "ring"), ("dma", "ring"), ("device", "mesh")] \
            if ring else [("device", "hd"), ("host", "hd"), ("dma", "hd")]
        for eng, sched in engines:
            buf = to_dev(x, dt)
            del_src = None
            gloo_amd.set_steps_engine(eng)
            try:
                if sched == "hd":
                    alg = gloo_amd.AllreduceHalvingDoubling(ctx, [buf], dtype=dt)
                else:
                    alg = gloo_amd.AllreduceRingChunked(ctx, [buf], schedule=sched, dtype=dt)
            finally:
                gloo_amd.set_steps_engine("auto")
            t0 = time.perf_counter()
            for it in range(2):
                if it:
                    buf.copy_(to_dev(x, dt))
                torch.cuda.synchronize()
                alg.run()
            ms = (time.perf_counter() - t0) * 1e3 / 2
            got = from_dev(buf, dt)
            ok = sha(got) == c["output_sha256"]
            if not ok and "sample_idx" not in c:
                bad.append((c["name"], sched, alg.engine(), "digest mismatch"))
            elif not ok:
                idx = np.array(c["sample_idx"])
                bits = np.ascontiguousarray(got).view(np.uint32 if got.itemsize == 4
                                                      else np.uint16)[idx]
                nbad = int((bits != np.array(c["sample"], dtype=bits.dtype)).sum())
                bad.append((c["name"], sched, alg.engine(), "sample mismatches", nbad))
            print("SCALE rank %d %s %s engine %s %.1f ms/run %s" % (
                rank, c["name"], sched, alg.engine(), ms, "ok" if ok else "MISMATCH"),
                flush=True)
            alg.close()
            del buf, del_src
            torch.cuda.empty_cache()
    store.set("done/%d" % rank, b"1")
    for r in range(size):
        store.get("done/%d" % r, timeout_ms=120000)
    print("IPC rank %d %s" % (rank, ctx.ipc_stats()), flush=True)
    ctx.close()
    if bad:
        print("MISMATCH rank", rank, bad[:10])
        sys.exit(1)
    print("OK")


if __name__ == "__main__":
    main()
