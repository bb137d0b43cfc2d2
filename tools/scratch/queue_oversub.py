#!/usr/bin/env python3
"""Diagnostic: do 8 rank processes sharing ONE GPU deadlock in the plan
kernel when the GPU's hardware queue slots are oversubscribed?

Round 3's full GPU suite once failed test_device_engine_multiprocess[8-devsteps]
(profiles/r7c_gpu_suite_failure.txt): rank 0 waited 20 s for a credit that
rank 1 never sent, though rank 0 had delivered the message (its flag read
through the mapping showed it).  The same test passed 3 of 3 times alone
(profiles/r7d_*).  In the suite the pytest parent holds a GPU context with
its own hardware queues; alone it holds none.  Each rank process opens up to
GPU_MAX_HW_QUEUES (default 4) hardware queues; when all processes' queues
exceed what the scheduler maps at once, some queue waits unmapped while the
peers' kernels spin on its flags.

Configurations (each: 8 rank processes, the ring plan kernel on a tiny buffer
run `iters` times with a 10 s context timeout):
  A  parent holds no GPU context, ranks default queues
  B  parent holds a context with `pstreams` busy streams, ranks default queues
  C  as B, ranks GPU_MAX_HW_QUEUES=1

    python tools/scratch/queue_oversub.py [iters] [pstreams] [ABC | P:q,P:q,...]
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rank_main(store_dir, rank, size, iters):
    sys.path.insert(0, ROOT)
    import torch
    import gloo_amd
    store = gloo_amd.rendezvous.FileStore(store_dir)
    ctx = gloo_amd.rendezvous.Context(rank, size, 0)
    ctx.setTimeout(10)
    ctx.connectFullMesh(store)
    # extra streams with work, as the executor's copy / staging streams and
    # torch's own would have (each may get a hardware queue of its own)
    side = [torch.cuda.Stream() for _ in range(3)]
    for s in side:
        with torch.cuda.stream(s):
            torch.ones(16, device="cuda").sum()
    buf = torch.ones(1, device="cuda")
    alg = gloo_amd.AllreduceRingChunked(ctx, [buf], schedule="ring")
    t0 = time.time()
    err = None
    done = 0
    try:
        for _ in range(iters):
            buf.fill_(1.0)
            torch.cuda.synchronize()
            alg.run()
            done += 1
            if buf.item() != size:
                err = "wrong result %r" % buf.item()
                break
    except Exception as e:  # noqa: BLE001
        err = "%s: %s" % (type(e).__name__, str(e)[:300])
    print(json.dumps({"rank": rank, "engine": alg.engine(), "done": done, "err": err,
                      "s": round(time.time() - t0, 2)}), flush=True)
    alg.close()
    return 0 if err is None else 1


def run_config(name, iters, parent_streams, rank_env, P=8):
    import torch  # noqa: F401
    keep = []
    if parent_streams:
        import torch
        for _ in range(parent_streams):
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                keep.append(torch.ones(1 << 20, device="cuda") * 2)
        torch.cuda.synchronize()
    with tempfile.TemporaryDirectory() as d:
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", **rank_env)
        t0 = time.time()
        procs = [subprocess.Popen([sys.executable, __file__, "rank", d, str(r), str(P), str(iters)],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(P)]
        outs = []
        for p in procs:
            o, _ = p.communicate(timeout=240)
            outs.append(o.decode(errors="replace"))
    res = []
    for o in outs:
        lines = [ln for ln in o.splitlines() if ln.startswith("{")]
        res.append(json.loads(lines[-1]) if lines else {"err": o[-300:]})
    ok = all(r.get("err") is None for r in res)
    print(json.dumps({"config": name, "P": P, "ok": ok, "wall_s": round(time.time() - t0, 1),
                      "parent_streams": parent_streams, "rank_env": rank_env,
                      "ranks": res}), flush=True)
    return ok


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "rank":
        return rank_main(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]))
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    pstreams = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    which = sys.argv[3] if len(sys.argv) > 3 else "ABC"
    if ":" in which:  # a sweep: "P:queues,P:queues,..." with the parent's streams busy
        for item in which.split(","):
            P, q = (int(x) for x in item.split(":"))
            env = {} if q == 4 else {"GPU_MAX_HW_QUEUES": str(q)}
            run_config("P%d_q%d" % (P, q), iters, pstreams, env, P=P)
        return 0
    if "A" in which:
        run_config("A", iters, 0, {})
    if "B" in which:
        run_config("B", iters, pstreams, {})
    if "C" in which:
        run_config("C", iters, pstreams, {"GPU_MAX_HW_QUEUES": "1"})
    return 0


if __name__ == "__main__":
    sys.exit(main())
