"""Host-memory endpoints fed from a socket: the reference's
path starts in host memory that a transport fills (gloo/transport/tcp/
pair.cc:385-451 receives into the registered buffer) and returns results the
same way.  Here each rank's host buffer is filled from a real TCP loopback
socket by a receiver thread that calls alg.feed() as bytes arrive, while the
rank runs alg.run_fed(): every 8 MiB piece is copied to the device as soon as
it is complete and each schedule step waits only for its own pieces.  The
result must be the reference's bits (oracle), done_ranges() must cover the
buffer, and a piece that never arrives must end in IoException."""
import socket
import threading

import numpy as np
import pytest

from helpers import case_inputs, run_ranks, same_bits
from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

PIECE = 1 << 20  # socket send size (bytes)


def socket_feeder(alg, buf, data, order="in_order"):
    """A loopback TCP connection: a sender thread writes `data`'s bytes (in
    `order`), the returned receiver thread recv_into()s them into `buf` and
    feeds the elements each recv completes."""
    es = buf.itemsize
    srv = socket.create_server(("127.0.0.1", 0))
    port = srv.getsockname()[1]
    raw = memoryview(np.ascontiguousarray(data).view(np.uint8))
    dst = memoryview(buf.view(np.uint8))
    nbytes = raw.nbytes
    pieces = [(o, min(PIECE, nbytes - o)) for o in range(0, nbytes, PIECE)]
    if order == "reversed":
        pieces = pieces[::-1]

    def send():
        with socket.create_connection(("127.0.0.1", port)) as c:
            for o, n in pieces:
                c.sendall(o.to_bytes(8, "little") + n.to_bytes(8, "little"))
                c.sendall(raw[o:o + n])

    def recv():
        conn, _ = srv.accept()
        with conn:
            for _ in range(len(pieces)):
                hdr = bytearray(16)
                got = 0
                while got < 16:
                    got += conn.recv_into(memoryview(hdr)[got:], 16 - got)
                o = int.from_bytes(hdr[:8], "little")
                n = int.from_bytes(hdr[8:], "little")
                got = 0
                while got < n:
                    k = conn.recv_into(dst[o + got:o + n], n - got)
                    assert k > 0
                    got += k
                    # feed the whole elements of this piece received so far
                lo, hi = o // es, (o + n) // es
                alg.feed(lo, hi - lo)
        srv.close()

    ts = [threading.Thread(target=send, daemon=True), threading.Thread(target=recv, daemon=True)]
    for t in ts:
        t.start()
    return ts


def fed_allreduce(algo, P, N, dtype=O.FLOAT32, order="in_order", runs=1, poll=None):
    """poll: per-rank lists that collect done_ranges() snapshots taken by a
    second thread while the fed runs are in flight (a consumer streaming
    finished ranges back out, what done_ranges() is for)."""
    import gloo_amd
    ins = case_inputs(P, N, dtype, 1, 0, seed=41)
    store = gloo_amd.rendezvous.HashStore()
    bufs = [np.zeros(N, dtype=O.NP_DTYPE[dtype]) for _ in range(P)]
    done = [None] * P

    def rank_fn(r):
        ctx = gloo_amd.rendezvous.Context(r, P, 0)
        ctx.setTimeout(60)
        ctx.connectFullMesh(store)
        dt = dtype if dtype in (O.FLOAT16, O.BFLOAT16) else None
        if algo == "halving_doubling":
            alg = gloo_amd.AllreduceHalvingDoubling(ctx, [bufs[r]], dtype=dt)
        else:
            alg = gloo_amd.AllreduceRingChunked(ctx, [bufs[r]], schedule="ring", dtype=dt)
        stop = threading.Event()

        def poller():
            while not stop.is_set():
                poll[r].append(alg.done_ranges())

        pt = threading.Thread(target=poller, daemon=True) if poll is not None else None
        if pt is not None:
            pt.start()
        try:
            for _ in range(runs):
                ts = socket_feeder(alg, bufs[r], ins[r][0], order)
                alg.run_fed()
                for t in ts:
                    t.join(60)
        finally:
            stop.set()
            if pt is not None:
                pt.join(60)
        done[r] = alg.done_ranges()
        alg.close()
        return True

    run_ranks(P, rank_fn, timeout=120)
    return bufs, done, ins


def covered(ranges, N):
    m = np.zeros(N, dtype=bool)
    for o, n in ranges:
        m[o:o + n] = True
    return bool(m.all())


@pytest.mark.parametrize("algo", ["ring_chunked", "halving_doubling"])
@pytest.mark.parametrize("P,N", [(1, 100003), (2, 3 << 20), (3, (5 << 20) + 7), (4, 1 << 22)])
def test_socket_fed_allreduce_vs_oracle(algo, P, N):
    bufs, done, ins = fed_allreduce(algo, P, N)
    code = O.HALVING_DOUBLING if algo == "halving_doubling" else O.RING_CHUNKED
    exp = O.allreduce(code, O.SUM, O.FLOAT32, ins)
    for r in range(P):
        assert same_bits(bufs[r], exp[r][0]), "rank %d" % r
        assert covered(done[r], N)


def test_socket_fed_out_of_order_and_repeated():
    """Pieces arriving back to front (a transport delivering out of order)
    and two fed runs on one instance."""
    P, N = 2, (3 << 20) + 5
    bufs, done, ins = fed_allreduce("ring_chunked", P, N, order="reversed", runs=2)
    exp = O.allreduce(O.RING_CHUNKED, O.SUM, O.FLOAT32, ins)
    for r in range(P):
        assert same_bits(bufs[r], exp[r][0])
        assert covered(done[r], N)


def test_socket_fed_float16():
    P, N = 2, (2 << 20) + 3
    bufs, done, ins = fed_allreduce("ring_chunked", P, N, dtype=O.FLOAT16)
    exp = O.allreduce(O.RING_CHUNKED, O.SUM, O.FLOAT16, ins)
    for r in range(P):
        assert same_bits(bufs[r], exp[r][0])


def test_unfed_piece_times_out():
    """A piece that never arrives: run_fed() raises IoException ("Timed out
    waiting for host data") after the context timeout instead of hanging."""
    import gloo_amd
    N = 3 << 20
    ctx = gloo_amd.rendezvous.Context(0, 1, 0)
    ctx.setTimeout(2)
    buf = np.zeros(N, dtype=np.float32)
    alg = gloo_amd.AllreduceRingChunked(ctx, [buf])
    alg.feed(0, N // 2)  # the second half never comes
    with pytest.raises(gloo_amd.IoException, match="host data"):
        alg.run_fed()
    alg.close()


@pytest.mark.parametrize("P", [1, 2, 3])
def test_done_ranges_polled_while_runs_are_in_flight(P):
    """A second thread polls done_ranges() without pause during the fed runs:
    ranges complete between the wrapper's calls into the C ABI (round 3's
    race), every snapshot must be well-formed ranges inside the
    buffer, and the final result exact and fully covered."""
    N = (3 << 20) + 11
    poll = [[] for _ in range(P)]
    bufs, done, ins = fed_allreduce("ring_chunked", P, N, runs=2, poll=poll)
    exp = O.allreduce(O.RING_CHUNKED, O.SUM, O.FLOAT32, ins)
    for r in range(P):
        assert same_bits(bufs[r], exp[r][0])
        assert covered(done[r], N)
        assert poll[r], "the poller never ran"
        for snap in poll[r]:
            for o, n in snap:
                assert 0 <= o and 0 < n and o + n <= N


@pytest.mark.parametrize("algo", ["ring_chunked", "halving_doubling"])
def test_socket_fed_through_bounce_block(algo):
    """A fed run whose buffer has no whole pinned mirror (the bounce block of
    executor_host.cc): H2D pieces are issued by the feeding thread while the
    run's thread copies finished ranges back through the block's other half,
    out-of-order pieces, two runs."""
    import gloo_amd
    gloo_amd.set_pinned_mirror_limit(4096)
    try:
        P, N = 3, (5 << 20) + 7
        bufs, done, ins = fed_allreduce(algo, P, N, order="reversed", runs=2)
    finally:
        gloo_amd.set_pinned_mirror_limit(0)
    code = O.HALVING_DOUBLING if algo == "halving_doubling" else O.RING_CHUNKED
    exp = O.allreduce(code, O.SUM, O.FLOAT32, ins)
    for r in range(P):
        assert same_bits(bufs[r], exp[r][0]), "rank %d" % r
        assert covered(done[r], N)
