"""Shared test helpers: golden fixtures, plan replay, thread-rank launcher."""
import hashlib
import json
import os
import threading

import numpy as np

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SEED = 1234


def sha(arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).view(np.uint8).tobytes())
    return h.hexdigest()


def load_allreduce_golden():
    with open(os.path.join(GOLDEN, "allreduce_golden.json")) as f:
        index = json.load(f)["cases"]
    data = np.load(os.path.join(GOLDEN, "allreduce_golden.npz"))
    return index, data


def load_ring_golden(which="ring"):
    """gloo::AllreduceRing<T> / AllreduceBcube<T> fixtures (make_golden.py
    ring / bcube): per-rank output digests (results may differ between
    ranks), full per-rank outputs for N <= 4099 under '<name>_r<rank>'."""
    with open(os.path.join(GOLDEN, "allreduce_%s_golden.json" % which)) as f:
        index = json.load(f)["cases"]
    data = np.load(os.path.join(GOLDEN, "allreduce_%s_golden.npz" % which))
    return index, data


def check_ring_against_golden(rec, data, outs):
    """outs: per rank, the list of its pointers' output arrays (the digest
    covers all of them, the stored array is the first)."""
    for r, row in enumerate(outs):
        assert sha(row) == rec["output_sha256"][r], "%s rank %d: digest" % (rec["name"], r)
        key = "%s_r%d" % (rec["name"], r)
        if key in data.files:
            assert np.array_equal(np.ascontiguousarray(row[0]).view(np.uint8),
                                  data[key].view(np.uint8)), key


def case_inputs(P, N, dtype, nptrs, kind, seed=SEED):
    ins = []
    for r in range(P):
        row = []
        for i in range(nptrs):
            if kind == 0:
                row.append(O.fill(dtype, N, 0, seed=seed, rank=r, ptr_index=i))
            elif kind == 1:
                row.append(O.fill(dtype, N, 1, stride=P * nptrs, val=r * nptrs + i))
            else:
                row.append(O.fill(dtype, N, 2, val=r))
        ins.append(row)
    return ins


def load_allreduce_fn_golden():
    with open(os.path.join(GOLDEN, "allreduce_fn_golden.json")) as f:
        index = json.load(f)["cases"]
    data = np.load(os.path.join(GOLDEN, "allreduce_fn_golden.npz"))
    return index, data


def fn_case_buffers(rec):
    """(inputs, outputs) per rank of a gloo::allreduce golden case, rebuilt
    exactly as tests/golden/make_golden.py made them."""
    P, N, dtype = rec["P"], rec["N"], rec["dtype"]
    nin, nout, kind = rec["nin"], rec["nout"], rec["kind"]
    if rec["out_init"] == "pattern":
        return [[] for _ in range(P)], case_inputs(P, N, dtype, nout, kind)
    ins = case_inputs(P, N, dtype, nin, kind)
    if rec["out_init"] == "zero":
        outs = [[np.zeros(N, dtype=O.NP_DTYPE[dtype]) for _ in range(nout)] for _ in range(P)]
    else:
        outs = [[O.fill(dtype, N, 0, seed=SEED + 1, rank=r, ptr_index=i) for i in range(nout)]
                for r in range(P)]
    return ins, outs


def check_against_golden(rec, data, out):
    """out: rank-0 result array of the case `rec`."""
    name = rec["name"]
    assert sha([out]) == rec["output_sha256"], "output checksum differs for " + name
    if name in data:
        assert np.array_equal(out.view(np.uint8), data[name].view(np.uint8))
    else:
        idx = data[name + "_idx"]
        assert np.array_equal(out[idx].view(np.uint8), data[name + "_sample"].view(np.uint8))


def same_bits(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint8),
                          np.ascontiguousarray(b).view(np.uint8))


# ---------------------------------------------------------------------------
# Replay of the product's step programs (glx_plan) on the host, with the
# executor's landing/credit rules: a message lands in the receiver's region
# when it is SENT (as a hipMemcpyPeerAsync does), and only after the credit
# for the previous message on that channel.  Any schedule bug that lets a
# message overwrite an unconsumed one, or reads a region before its message
# arrived, shows up as a result that differs from the oracle.
# ---------------------------------------------------------------------------
def replay_plans(plans, op, dtype, inputs):
    P = len(plans)
    data = [np.array(inputs[r], copy=True) for r in range(P)]
    scratch = [np.zeros(max(pl[1], 1), dtype=data[0].dtype) for pl in plans]
    pc = [0] * P
    sent = {}       # (src, dst, tag) -> messages sent
    delivered = {}  # (src, dst, tag) -> messages landed
    consumed = {}   # (src, dst, tag) -> messages released
    received = {}
    blocked_rounds = 0
    while True:
        progress = False
        done = True
        for r in range(P):
            steps = plans[r][0]
            while pc[r] < len(steps):
                kind, peer, tag, off, ln, boff, dst_off, _ = steps[pc[r]]
                if kind == 0:  # SEND
                    key = (r, peer, tag)
                    n = sent.get(key, 0) + 1
                    if consumed.get(key, 0) < n - 1:
                        break  # no credit yet
                    scratch[peer][dst_off:dst_off + ln] = data[r][off:off + ln]
                    sent[key] = n
                    delivered[key] = n
                elif kind == 1:  # RECV
                    key = (peer, r, tag)
                    n = received.get(key, 0) + 1
                    if delivered.get(key, 0) < n:
                        break
                    received[key] = n
                elif kind == 2:  # REDUCE
                    data[r][off:off + ln] = O.reduce(op, dtype, data[r][off:off + ln],
                                                     scratch[r][boff:boff + ln])
                elif kind == 3:  # COPY
                    data[r][off:off + ln] = scratch[r][boff:boff + ln]
                elif kind == 5:  # FOLD: acc = s0; acc = op(s_k, acc) (or op(acc, s_k))
                    srcs = plans[r][2][boff]
                    left = bool(steps[pc[r]][7] & 1)
                    whole = bool(steps[pc[r]][7] & 2)  # whole-buffer source regions

                    def val(reg, r=r, off=off, ln=ln, whole=whole):
                        if reg == -1:
                            return np.array(data[r][off:off + ln], copy=True)
                        at = reg + off if whole else reg
                        return scratch[r][at:at + ln]
                    acc = np.array(val(srcs[0]), copy=True)
                    for reg in srcs[1:]:
                        acc = (O.reduce(op, dtype, acc, val(reg)) if left
                               else O.reduce(op, dtype, val(reg), acc))
                    data[r][off:off + ln] = acc
                elif kind == 4:  # RELEASE
                    key = (peer, r, tag)
                    consumed[key] = consumed.get(key, 0) + 1
                pc[r] += 1
                progress = True
            if pc[r] < len(steps):
                done = False
        if done:
            break
        if not progress:
            blocked_rounds += 1
            raise AssertionError("plan replay deadlocked at pcs %s" % pc)
    return data


def run_ranks(P, fn, timeout=120):
    """Run fn(rank) on P threads (the reference tests' topology,
    gloo/test/base_test.h:91-166); re-raise the first failure."""
    errors = [None] * P
    results = [None] * P

    def body(r):
        try:
            results[r] = fn(r)
        except BaseException as e:  # noqa: BLE001
            errors[r] = e

    threads = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(P)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout)
        if t.is_alive():
            raise TimeoutError("rank thread did not finish within %ss" % timeout)
    for e in errors:
        if e is not None:
            raise e
    return results


def rank_env(P, device_engines="shared"):
    """Environment of P rank processes sharing the box's one GPU: a
    rehearsal of the node's one-process-per-GPU run.  By default the ranks
    opt in to the device engines on the shared GPU (GLOO_AMD_DEVICE_ENGINES=
    shared: the tests queue no other GPU work ahead of a collective), which
    the library's automatic mode gives only to ranks with a GPU of their own
    (DESIGN.md 5a, 9); device_engines=None keeps the automatic mode.  Device
    engines need every rank's kernel running at once; the GPU's scheduler
    maps a bounded number of hardware queues and time-slices the rest, so
    above 4 ranks each process keeps to one queue (the shared mode's budget,
    HipPlanExecutor::kSharedQueueBudget: ranks x (queues + 1) <= 20; 8 ranks
    x 2 queues measured time-sliced, profiles/r7g_queue_sweep.txt)."""
    import os
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.setdefault("PYTHONFAULTHANDLER", "1")  # a crashing rank prints its stacks
    env.pop("GLOO_AMD_DEVICE_ENGINES", None)
    if device_engines is not None:
        env["GLOO_AMD_DEVICE_ENGINES"] = device_engines
    if P > 4:
        env["GPU_MAX_HW_QUEUES"] = "1"
    return env
