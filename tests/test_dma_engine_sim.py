"""CPU: the DMA steps engine's enqueue order and its deadlock rule, simulated
(executor.cc exchangeDma).

Each rank's compiled step program (glx_plan) becomes the packets exchangeDma
enqueues -- copies, reduce / copy / fold launches, one-wave flag kernels
(waits and signals on flag words), and, for host buffers, the copy-back
stream's event waits after every step's launch -- in the order it enqueues
them.  Every stream of a rank is mapped onto one of Q hardware queues (HIP
shares queues between a process's streams once it has more streams than
GPU_MAX_HW_QUEUES); a queue runs its packets in enqueue order, a flag kernel
holds its queue until its waits are met, copies and launches complete at the
head.  Signals only raise words and waits only ask for ``>=``, so the greedy
run below reaches the one maximal state: it stalls exactly when the rule
deadlocks.

* The rule in the product (one pending list, flushed whenever the next op
  or enqueue is for another stream) finishes every rank for every mapping of
  its streams onto 1-4 queues, ring / halving-doubling / bcube / function-
  style ring at P = 2..8, two runs back to back.
* The first version (a copy's signals held in that stream's list until its
  next copy) is caught: with a hardware queue shared by the compute and copy
  streams it stalls -- the cycle the staged GPU test hit (P = 2, "receive step
  13"), while with a queue per stream it finishes.
"""
import itertools
import random

import pytest

import gloo_amd

SEND, RECV, REDUCE, COPY, RELEASE, FOLD = range(6)
MAX_OPS = 8  # glx::kFlagOpsMax


def packets(r, steps, runs, staged, rule):
    """The packets rank r enqueues over `runs` runs, in enqueue order:
    ("flag", stream, [(kind, word, value)]), ("work", stream),
    ("event", stream, id), ("evwait", stream, id).  Words are global keys:
    (rank, "deliv", peer, tag), (rank, "credit", peer, tag), (rank, "mark"),
    (rank, "done", stream)."""
    out = []
    sent, received, consumed, copies, waited = {}, {}, {}, {}, {}
    marks = [0]
    ev = [0]
    pend = []  # rule "ordered": [(stream, op)], one stream at a time
    per = {}   # rule "deferred": stream -> [op]

    def flush(stream=None):
        if rule == "ordered":
            if pend:
                out.append(("flag", pend[0][0], [o for _, o in pend]))
                pend.clear()
        else:
            ops = per.get(stream)
            if ops:
                out.append(("flag", stream, list(ops)))
                ops.clear()

    def op(stream, o):
        if rule == "ordered":
            if pend and (pend[0][0] != stream or len(pend) == MAX_OPS):
                flush()
            pend.append((stream, o))
        else:
            ops = per.setdefault(stream, [])
            if len(ops) == MAX_OPS:
                flush(stream)
            ops.append(o)

    def copy_stream(peer, tag):
        # the product: one per channel; the first version: one per peer
        return ("copy", peer, tag) if rule == "ordered" else ("copy", peer)

    def launch(step):
        """flush (the compute stream's list in the first version), the
        launch, then the copy-back of its final values (host buffers)"""
        flush("compute")
        out.append(("work", "compute"))
        if staged:
            flush("compute")
            ev[0] += 1
            out.append(("event", "compute", (r, ev[0])))
            out.append(("evwait", "d2h", (r, ev[0])))
            out.append(("work", "d2h"))

    for _ in range(runs):
        inflight = []
        since_mark = True
        i = 0
        while i < len(steps):
            kind, peer, tag, off, ln = steps[i][:5]
            if kind == SEND:
                n = sent[(peer, tag)] = sent.get((peer, tag), 0) + 1
                cs = copy_stream(peer, tag)
                if since_mark:
                    marks[0] += 1
                    op("compute", ("S", (r, "mark"), marks[0]))
                    since_mark = False
                if waited.get(cs) != marks[0]:
                    op(cs, ("W", (r, "mark"), marks[0]))
                    waited[cs] = marks[0]
                if n > 1:
                    op(cs, ("W", (r, "credit", peer, tag), n - 1))
                if staged and rule == "ordered":
                    flush()  # the H2D wait (pieces issued before the run)
                flush(cs)
                out.append(("work", cs))
                copies[cs] = copies.get(cs, 0) + 1
                op(cs, ("S", (peer, "deliv", r, tag), n))
                op(cs, ("S", (r, "done", cs), copies[cs]))
                inflight.append((off, ln, cs, copies[cs]))
            elif kind == RECV:
                received[(peer, tag)] = received.get((peer, tag), 0) + 1
                op("compute", ("W", (r, "deliv", peer, tag), received[(peer, tag)]))
            elif kind in (REDUCE, COPY, FOLD):
                last = i
                if kind == FOLD:  # consecutive FOLDs of one kind: one launch
                    while (last + 1 < len(steps) and steps[last + 1][0] == FOLD
                           and steps[last + 1][7] == steps[i][7]):
                        last += 1
                for q in range(i, last + 1):
                    o, n_ = steps[q][3], steps[q][4]
                    keep = []
                    for f in inflight:
                        if f[0] < o + n_ and o < f[0] + f[1]:
                            op("compute", ("W", (r, "done", f[2]), f[3]))
                        else:
                            keep.append(f)
                    inflight = keep
                    if staged and rule == "ordered":
                        flush()
                launch(i)
                since_mark = True
                i = last
            elif kind == RELEASE:
                consumed[(peer, tag)] = consumed.get((peer, tag), 0) + 1
                op("compute", ("S", (peer, "credit", r, tag), consumed[(peer, tag)]))
            i += 1
        for cs in sorted({k for k in copies}, key=str):
            flush(cs)
            op("compute", ("W", (r, "done", cs), copies[cs]))
        flush("compute")
        flush()
    return out


def streams_of(pk):
    return sorted({p[1] for p in pk}, key=str)


def run_ranks(pks, queue_of):
    """pks[r]: rank r's packets; queue_of[r]: stream -> hardware queue.
    Returns the ranks left with packets when no queue can move (empty: all
    finished)."""
    words = {}
    fired = set()
    queues = []
    for r, pk in enumerate(pks):
        qs = {}
        for p in pk:
            qs.setdefault(queue_of[r][p[1]], []).append(p)
        queues.append({q: [list(x), 0] for q, x in qs.items()})  # packets, op index
    moved = True
    while moved:
        moved = False
        for r in range(len(pks)):
            for q, state in queues[r].items():
                pk, k = state
                while pk:
                    p = pk[0]
                    if p[0] == "flag":
                        ops = p[2]
                        while k < len(ops):
                            kind, w, v = ops[k]
                            if kind == "S":
                                words[w] = max(words.get(w, 0), v)
                            elif words.get(w, 0) < v:
                                break
                            k += 1
                            moved = True
                        if k < len(ops):
                            break
                        k = 0
                    elif p[0] == "event":
                        fired.add(p[2])
                    elif p[0] == "evwait" and p[2] not in fired:
                        break
                    pk.pop(0)
                    moved = True
                state[1] = k
    return [r for r in range(len(pks)) if any(s[0] for s in queues[r].values())]


def mappings(streams, Q, rng, count):
    """`count` random maps of the streams onto Q queues, plus the extremes:
    one queue for all, and (if Q allows) a queue each."""
    out = [{s: 0 for s in streams}]
    if len(streams) <= Q:
        out.append({s: i for i, s in enumerate(streams)})
    for _ in range(count):
        out.append({s: rng.randrange(Q) for s in streams})
    return out


CASES = [("ring_chunked", P, n) for P in (2, 3, 4, 5, 8) for n in (1 << 16, 100003)] + \
        [("halving_doubling", P, n) for P in (2, 3, 4, 6, 8) for n in (1 << 16, 99991)] + \
        [("bcube", P, 1 << 16) for P in (2, 4, 8)] + \
        [("fn_ring", P, 1 << 16) for P in (2, 4, 8)]


@pytest.mark.parametrize("algo,P,N", CASES)
@pytest.mark.parametrize("staged", [False, True])
def test_program_order_rule_never_stalls(algo, P, N, staged):
    progs = [gloo_amd.plan(algo, r, P, N)[0] for r in range(P)]
    pks = [packets(r, progs[r], 2, staged, "ordered") for r in range(P)]
    rng = random.Random(hash((algo, P, N, staged)) & 0xffff)
    for Q in (1, 2, 3, 4):
        per_rank = [mappings(streams_of(pk), Q, rng, 6) for pk in pks]
        for choice in range(len(per_rank[0])):
            qmap = [m[min(choice, len(m) - 1)] for m in per_rank]
            stuck = run_ranks(pks, qmap)
            assert not stuck, (algo, P, N, staged, Q, qmap, stuck)


def test_deferred_copy_signals_stall_under_a_shared_queue():
    """The first version's cycle (staged host buffers, P = 2, ring): found
    when the compute and copy streams share a hardware queue; a queue per
    stream hides it."""
    P, N = 2, 65536
    progs = [gloo_amd.plan("ring_chunked", r, P, N)[0] for r in range(P)]
    pks = [packets(r, progs[r], 1, True, "deferred") for r in range(P)]
    streams = streams_of(pks[0])
    assert len(streams) == 3  # compute, the copy stream to the peer, the copy-back stream
    own = [{s: i for i, s in enumerate(streams_of(pk))} for pk in pks]
    assert not run_ranks(pks, own)
    shared = [{s: (0 if s != "d2h" else 1) for s in streams_of(pk)} for pk in pks]
    assert run_ranks(pks, shared) == [0, 1]
    # the product's rule on the same shapes
    pks = [packets(r, progs[r], 1, True, "ordered") for r in range(P)]
    for qmap_r in itertools.product(range(2), repeat=len(streams_of(pks[0]))):
        qmap = [dict(zip(streams_of(pk), qmap_r)) for pk in pks]
        assert not run_ranks(pks, qmap)


@pytest.mark.parametrize("algo,P,N", [("ring_chunked", 2, 20000), ("ring_chunked", 4, 40000),
                                      ("halving_doubling", 2, 20000),
                                      ("halving_doubling", 4, 40000), ("fn_bcube", 4, 40000)])
@pytest.mark.parametrize("staged", [False, True])
def test_program_order_rule_with_split_messages(algo, P, N, staged):
    """split programs (4 KiB pieces, one channel per piece
    index) under the DMA steps engine's enqueue rule and every mapping of its
    streams onto hardware queues: no stall."""
    gloo_amd.set_max_message_bytes(4096)
    try:
        progs = [gloo_amd.plan(algo, r, P, N)[0] for r in range(P)]
    finally:
        gloo_amd.set_max_message_bytes(0)
    assert max(s[4] for pr in progs for s in pr if s[0] in (0, 1)) <= 1024
    pks = [packets(r, progs[r], 2, staged, "ordered") for r in range(P)]
    rng = random.Random(hash((algo, P, N, staged, "split")) & 0xffff)
    for Q in (1, 2, 3, 4):
        per_rank = [mappings(streams_of(pk), Q, rng, 4) for pk in pks]
        for choice in range(len(per_rank[0])):
            qmap = [m[min(choice, len(m) - 1)] for m in per_rank]
            stuck = run_ranks(pks, qmap)
            assert not stuck, (algo, P, N, staged, Q, qmap, stuck)


@pytest.mark.parametrize("algo,P,N", [("ring_chunked", 2, 20000), ("ring_chunked", 4, 40000),
                                      ("ring_chunked", 8, 80000),
                                      ("halving_doubling", 4, 40000)])
def test_program_order_rule_with_pipelined_messages(algo, P, N):
    """the pipelined programs (4 KiB pieces, reduce-and-forward
    per piece) under the DMA steps engine's enqueue rule: no stall on any
    mapping of its streams onto 1-4 hardware queues."""
    gloo_amd.set_pipeline_bytes(4096)
    try:
        progs = [gloo_amd.plan(algo, r, P, N)[0] for r in range(P)]
    finally:
        gloo_amd.set_pipeline_bytes(0)
    pks = [packets(r, progs[r], 2, False, "ordered") for r in range(P)]
    rng = random.Random(hash((algo, P, N, "pipe")) & 0xffff)
    for Q in (1, 2, 3, 4):
        per_rank = [mappings(streams_of(pk), Q, rng, 4) for pk in pks]
        for choice in range(len(per_rank[0])):
            qmap = [m[min(choice, len(m) - 1)] for m in per_rank]
            stuck = run_ranks(pks, qmap)
            assert not stuck, (algo, P, N, Q, qmap, stuck)
