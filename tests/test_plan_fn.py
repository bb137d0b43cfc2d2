"""Function-style allreduce schedules (gloo/allreduce.cc ring and bcube):
the product's step programs (glx_plan_ex) replayed on the host with the
executor's landing/credit rules, against the oracle's restatement of
gloo::allreduce (itself pinned to the compiled reference in test_oracle_fn.py).
No GPU needed."""
import numpy as np
import pytest

from gloo_amd import algorithms as A
from helpers import replay_plans, same_bits
from oracle import oracle as O

CASES = [(P, N) for P in (2, 3, 4, 5, 7, 8) for N in (1, 7, 100, 1000, 4099, 20000)]
DT_OPS = [(O.FLOAT32, O.SUM), (O.INT32, O.SUM), (O.FLOAT16, O.SUM), (O.FLOAT16, O.MAX),
          (O.FLOAT32, O.MIN), (O.FLOAT64, O.PRODUCT)]
ESIZE = {O.FLOAT32: 4, O.INT32: 4, O.FLOAT16: 2, O.FLOAT64: 8}


def _inputs(P, N, dtype):
    return [O.fill(dtype, N, 0, seed=5, rank=r) for r in range(P)]


def _replay(algo, P, N, dtype, op, max_seg, piece):
    plans = [A.plan(algo, r, P, N, with_folds=True, esize=ESIZE[dtype],
                    max_segment_size=max_seg, min_piece_bytes=piece) for r in range(P)]
    return replay_plans(plans, op, dtype, _inputs(P, N, dtype))


def _oracle(algo_code, P, N, dtype, op, max_seg):
    outs = O.allreduce_fn(algo_code, op, dtype, [[] for _ in range(P)],
                          [[x] for x in _inputs(P, N, dtype)], max_seg)
    return [o[0] for o in outs]


@pytest.mark.parametrize("P,N", CASES)
@pytest.mark.parametrize("dtype,op", DT_OPS)
@pytest.mark.parametrize("max_seg", [128, 0])
def test_fn_ring_plan_matches_oracle(P, N, dtype, op, max_seg):
    exp = _oracle(O.FN_RING, P, N, dtype, op, max_seg)
    # the reference's own segments, device-sized pieces, and tiny pieces
    for piece in (0, A.DEFAULT_MIN_PIECE_BYTES, 256):
        got = _replay("fn_ring", P, N, dtype, op, max_seg, piece)
        for r in range(P):
            assert same_bits(got[r], exp[r]), (piece, r)


@pytest.mark.parametrize("P,N", CASES)
@pytest.mark.parametrize("dtype,op", DT_OPS)
@pytest.mark.parametrize("max_seg", [128, 0])
def test_fn_ring_mesh_plan_is_bit_identical(P, N, dtype, op, max_seg):
    exp = _oracle(O.FN_RING, P, N, dtype, op, max_seg)
    got = _replay("fn_ring_mesh", P, N, dtype, op, max_seg, 0)
    for r in range(P):
        assert same_bits(got[r], exp[r]), r


@pytest.mark.parametrize("P,N", CASES + [(6, 1000), (9, 1000), (12, 999), (16, 64)])
@pytest.mark.parametrize("dtype,op", DT_OPS)
def test_fn_bcube_plan_matches_oracle(P, N, dtype, op):
    exp = _oracle(O.FN_BCUBE, P, N, dtype, op, 0)
    got = _replay("fn_bcube", P, N, dtype, op, 0, 0)
    for r in range(P):
        assert same_bits(got[r], exp[r]), r


def test_fn_ring_traffic_is_the_ring_volume():
    P, N = 8, 1 << 20
    for r in range(P):
        steps, _ = A.plan("fn_ring", r, P, N)
        sent = sum(s[4] for s in steps if s[0] == 0)
        assert sent == 2 * (P - 1) * N // P


def test_fn_ring_pieces_respect_min_piece_bytes():
    P, N = 8, 64 << 20  # 256 MiB fp32
    steps, scratch = A.plan("fn_ring", 0, P, N)
    lens = {s[4] for s in steps if s[0] == 0}
    assert min(lens) * 4 >= A.DEFAULT_MIN_PIECE_BYTES
    # two receive regions per phase, each one piece (+ landing padding)
    assert scratch == 4 * (max(lens) + 32)


def test_fn_bcube_uses_log_steps_for_power_of_two():
    steps, _ = A.plan("fn_bcube", 0, 8, 1 << 16)
    peers = [s[1] for s in steps if s[0] == 0]
    assert peers == [1, 2, 4, 4, 2, 1]
