"""CPU: messages split into pieces (plan.h splitMessages).

Every message above glx_set_max_message_bytes goes as consecutive pieces,
each a message of its own landing in a receive region of its own, so no block
another process imports reaches the 2 GiB at which the HIP runtime's IPC
import hangs, at any count the reference accepts.  Here the threshold is
lowered to 4 KiB and the split programs -- exactly what the executor runs --
are replayed with the executor's landing and credit rules (helpers.
replay_plans: a SEND waits for the release of the channel's previous
message): every schedule must finish (no credit cycle) and reproduce the
oracle bit for bit, because splitting changes no per-element reduction chain.
"""
import numpy as np
import pytest

import gloo_amd
from helpers import case_inputs, replay_plans, same_bits
from oracle import oracle as O

SMALL = 4096  # bytes per piece in these tests


@pytest.fixture
def small_messages():
    gloo_amd.set_max_message_bytes(SMALL)
    try:
        yield SMALL
    finally:
        gloo_amd.set_max_message_bytes(0)
    assert gloo_amd.max_message_bytes() == 512 << 20


CLASS = {"ring_chunked": O.RING_CHUNKED, "halving_doubling": O.HALVING_DOUBLING,
         "ring_chunked_mesh": O.RING_CHUNKED}


@pytest.mark.parametrize("name", sorted(CLASS))
@pytest.mark.parametrize("P", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("N", [1000, 4099, 65537])
@pytest.mark.parametrize("dtype,op", [(O.FLOAT32, O.SUM), (O.FLOAT16, O.SUM),
                                      (O.INT8, O.MAX), (O.FLOAT64, O.PRODUCT)])
def test_split_class_programs_match_the_oracle(small_messages, name, P, N, dtype, op):
    es = np.dtype(O.NP_DTYPE[dtype]).itemsize
    M = SMALL // es
    plans = [gloo_amd.plan(name, r, P, N, with_folds=True, esize=es) for r in range(P)]
    msgs = [s[4] for pl in plans for s in pl[0] if s[0] in (0, 1)]
    assert max(msgs) <= M, "a message above the threshold was not split"
    gloo_amd.set_max_message_bytes(1 << 40)
    try:
        whole = [gloo_amd.plan(name, r, P, N, esize=es) for r in range(P)]
    finally:
        gloo_amd.set_max_message_bytes(SMALL)
    before = max(s[4] for pl in whole for s in pl[0] if s[0] in (0, 1))
    if before > M:  # it was split: more messages, the same bytes
        assert len(msgs) > sum(1 for pl in whole for s in pl[0] if s[0] in (0, 1))
    assert (sum(s[4] for pl in plans for s in pl[0] if s[0] == 0)
            == sum(s[4] for pl in whole for s in pl[0] if s[0] == 0))
    ins = case_inputs(P, N, dtype, 1, 0, seed=P * 31 + N % 97)
    got = replay_plans(plans, op, dtype, [ins[r][0] for r in range(P)])
    exp = O.allreduce(CLASS[name], op, dtype, ins)
    for r in range(P):
        assert same_bits(got[r], exp[r][0]), "rank %d" % r


@pytest.mark.parametrize("name,code", [("fn_ring", O.FN_RING), ("fn_bcube", O.FN_BCUBE),
                                       ("fn_ring_mesh", O.FN_RING)])
@pytest.mark.parametrize("P", [2, 3, 4, 6, 8])
@pytest.mark.parametrize("N", [4099, 65537])
def test_split_function_style_programs_match_the_oracle(small_messages, name, code, P, N):
    dtype, op = O.FLOAT32, O.SUM
    plans = [gloo_amd.plan(name, r, P, N, with_folds=True, esize=4,
                           max_segment_size=64 << 10, min_piece_bytes=64 << 10)
             for r in range(P)]
    assert max(s[4] for pl in plans for s in pl[0] if s[0] in (0, 1)) <= SMALL // 4
    ins = case_inputs(P, N, dtype, 1, 0, seed=7 * P + 1)
    got = replay_plans(plans, op, dtype, [ins[r][0] for r in range(P)])
    exp = O.allreduce_fn(code, op, dtype, [[] for _ in range(P)], ins,
                         max_segment_size=64 << 10)
    for r in range(P):
        assert same_bits(got[r][0] if isinstance(got[r], list) else got[r], exp[r][0]), r


def test_whole_buffer_folds_stay_whole(small_messages):
    """AllreduceRing and the replicated schedules fold whole-buffer messages
    (kFoldWhole): they are left as they are (plan.h)."""
    for name in ("ring", "ring_chunked_repl"):
        steps, _ = gloo_amd.plan(name, 0, 4, 65537)
        assert max(s[4] for s in steps if s[0] in (0, 1)) == 65537


def test_max_message_bytes_setter_rejects_tiny_values():
    with pytest.raises(gloo_amd.EnforceNotMet):
        gloo_amd.set_max_message_bytes(100)
    with pytest.raises(gloo_amd.EnforceNotMet):
        gloo_amd.set_max_message_bytes(-1)
    assert gloo_amd.max_message_bytes() == 512 << 20


def test_huge_threshold_leaves_every_message_whole():
    """The executor compiles every rank's unsplit program (threshold 2^62) to
    decide whether the one- and two-shot kernels may run: the piece count
    must not overflow there (it once did, and the two-shot ran a split plan)."""
    gloo_amd.set_max_message_bytes((1 << 63) - 1)  # the executor's own probe value
    try:
        for es in (1, 2, 4):  # small buffers too: no (q + 1) * M overflow
            st = gloo_amd.plan("ring_chunked_mesh", 0, 2, 4099, esize=es)[0]
            assert max(s[4] for s in st if s[0] in (0, 1)) == 2050
        n = (1 << 31) - 1
        for name, es in (("ring_chunked_mesh", 1), ("ring_chunked_mesh", 2),
                         ("halving_doubling", 8), ("ring_chunked", 2)):
            whole = [s for s in gloo_amd.plan(name, 0, 2, n, esize=es)[0] if s[0] in (0, 1)]
            assert whole and min(s[4] for s in whole) > 0
            assert max(s[4] for s in whole) >= n // 4
    finally:
        gloo_amd.set_max_message_bytes(0)


@pytest.fixture
def pipelined():
    gloo_amd.set_pipeline_bytes(SMALL)
    try:
        yield SMALL
    finally:
        gloo_amd.set_pipeline_bytes(0)
    assert gloo_amd.pipeline_bytes() == 0


@pytest.mark.parametrize("name", sorted(CLASS))
@pytest.mark.parametrize("P", [2, 3, 4, 8])
@pytest.mark.parametrize("N", [4099, 65537])
@pytest.mark.parametrize("dtype,op", [(O.FLOAT32, O.SUM), (O.FLOAT16, O.SUM), (O.INT8, O.MAX)])
def test_pipelined_programs_match_the_oracle(pipelined, name, P, N, dtype, op):
    """pipelining below chunk granularity (glx_set_pipeline_bytes,
    splitMessages with forward): pieces of 4 KiB, the ring's reduce-and-forward
    (and the mesh's result sends) per piece -- no credit cycle, the oracle's
    bits."""
    es = np.dtype(O.NP_DTYPE[dtype]).itemsize
    plans = [gloo_amd.plan(name, r, P, N, with_folds=True, esize=es) for r in range(P)]
    assert max(s[4] for pl in plans for s in pl[0] if s[0] in (0, 1)) <= SMALL // es
    if name == "ring_chunked":
        # a forward right after each piece's RELEASE: RECV, REDUCE, RELEASE, SEND
        st = plans[0][0]
        fwd = [i for i in range(3, len(st)) if st[i][0] == 0 and st[i - 1][0] == 4
               and st[i - 2][0] == 2 and st[i][3] == st[i - 2][3] and st[i][4] == st[i - 2][4]]
        assert len(fwd) >= 2
    ins = case_inputs(P, N, dtype, 1, 0, seed=P * 13 + N % 89)
    got = replay_plans(plans, op, dtype, [ins[r][0] for r in range(P)])
    exp = O.allreduce(CLASS[name], op, dtype, ins)
    for r in range(P):
        assert same_bits(got[r], exp[r][0]), "rank %d" % r
