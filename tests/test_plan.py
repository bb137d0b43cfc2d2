"""CPU: the product's step programs (glx_plan -- exactly what the GPU executor
runs) replayed on the host with the executor's landing/credit rules must
reproduce the oracle bit for bit."""
import numpy as np
import pytest

import gloo_amd
from helpers import case_inputs, replay_plans, same_bits
from oracle import oracle as O

NAMES = {O.RING_CHUNKED: "ring_chunked", O.HALVING_DOUBLING: "halving_doubling"}


@pytest.mark.parametrize("algo", [O.RING_CHUNKED, O.HALVING_DOUBLING],
                         ids=["ring_chunked", "halving_doubling"])
@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 6, 7, 8, 9, 13, 16])
@pytest.mark.parametrize("N", [0, 1, 64, 255, 256, 1000, 4099])
@pytest.mark.parametrize("op", [O.SUM, O.MAX])
def test_plan_replay_matches_oracle(algo, P, N, op):
    ins = case_inputs(P, N, O.FLOAT32, 1, 0, seed=99)
    plans = [gloo_amd.plan(NAMES[algo], r, P, N) for r in range(P)]
    got = replay_plans(plans, op, O.FLOAT32, [ins[r][0] for r in range(P)])
    exp = O.allreduce(algo, op, O.FLOAT32, ins)
    for r in range(P):
        assert same_bits(got[r], exp[r][0]), "rank %d" % r


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 7, 8, 9, 16, 17])
@pytest.mark.parametrize("N", [0, 1, 255, 256, 1000, 4099, 65537])
@pytest.mark.parametrize("dtype,op", [(O.FLOAT32, O.SUM), (O.FLOAT32, O.MAX),
                                      (O.FLOAT32, O.MIN), (O.FLOAT16, O.SUM),
                                      (O.FLOAT16, O.PRODUCT), (O.INT32, O.PRODUCT)])
def test_mesh_schedule_is_bit_identical_to_ring_chunked(P, N, dtype, op):
    """The mesh schedule folds each chunk pair's chain in one pass with the
    ring's operand order, so it must reproduce AllreduceRingChunked exactly
    (fp32 sum rounding, max/min NaN/signed-zero choices, the fp16 quirk)."""
    ins = case_inputs(P, N, dtype, 1, 0, seed=123)
    if dtype == O.FLOAT32 and N > 10:
        for r in range(P):  # signed zeros and NaNs exercise max/min operand order
            ins[r][0][3] = -0.0 if r % 2 else 0.0
            ins[r][0][7] = np.nan if r == 1 else ins[r][0][7]
    plans = [gloo_amd.plan("ring_chunked_mesh", r, P, N, with_folds=True) for r in range(P)]
    got = replay_plans(plans, op, dtype, [ins[r][0] for r in range(P)])
    exp = O.allreduce(O.RING_CHUNKED, op, dtype, ins)
    for r in range(P):
        assert same_bits(got[r], exp[r][0]), "rank %d" % r


@pytest.mark.parametrize("P", [2, 4, 8])
def test_mesh_plan_traffic(P):
    """Per peer link: 2*S/P bytes (vs the ring's 2(P-1)/P * S over one link)."""
    N = 2 * P * 1024
    steps, _ = gloo_amd.plan("ring_chunked_mesh", 0, P, N)
    sends = [s for s in steps if s[0] == 0]
    per_peer = {}
    for s in sends:
        per_peer[s[1]] = per_peer.get(s[1], 0) + s[4]
    assert len(per_peer) == P - 1
    assert all(v == 2 * N // P for v in per_peer.values())


@pytest.mark.parametrize("P", [2, 4, 8])
def test_ring_plan_traffic(P):
    """4P-4 chunk sends per rank, 1.75*S link bytes at P=8."""
    N = 16 * P * 1000
    steps, _ = gloo_amd.plan("ring_chunked", 0, P, N)
    sends = [s for s in steps if s[0] == 0]
    assert len(sends) == 4 * P - 4
    assert sum(s[4] for s in sends) == (4 * P - 4) * N // (2 * P)


@pytest.mark.parametrize("P", [2, 4, 8])
def test_hd_plan_traffic(P):
    N = 1 << 16
    steps, _ = gloo_amd.plan("halving_doubling", 0, P, N)
    assert sum(s[4] for s in steps if s[0] == 0) == 2 * N * (P - 1) // P


def test_plan_rejects_bad_geometry():
    with pytest.raises(gloo_amd.EnforceNotMet):
        gloo_amd.plan("ring_chunked", 3, 2, 10)


# ---------------------------------------------------------------------------
# Host-memory staging (glx_plan_stage): every element copied in exactly once,
# copied back exactly once after its final write, pieces in first-use order.
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("algo", ["ring_chunked", "halving_doubling", "ring_chunked_mesh",
                                  "fn_ring", "fn_ring_mesh", "fn_bcube"])
@pytest.mark.parametrize("P,N", [(1, 1000), (2, 1), (2, 1000), (3, 4099), (5, 100003),
                                 (8, 1 << 16), (8, 4 << 20)])
def test_stage_plan_covers_each_element_once(algo, P, N):
    from gloo_amd import algorithms as A
    for r in range(P):
        steps, _ = A.plan(algo, r, P, N)
        h2d, d2h = A.stage_plan(algo, r, P, N, max_piece=1 << 18)
        cover = np.zeros(N, np.int32)
        for off, ln in h2d:
            assert 0 < ln <= 1 << 18
            cover[off:off + ln] += 1
        assert (cover == 1).all()
        back = np.zeros(N, np.int32)
        last_write = np.full(N, -1, np.int64)
        for i, st in enumerate(steps):
            if st[0] in (2, 3, 5) and st[4] > 0:
                last_write[st[3]:st[3] + st[4]] = i
        for step, off, ln in d2h:
            back[off:off + ln] += 1
            # copied back right after the step that writes the final value
            assert (last_write[off:off + ln] == step).all()
        assert (back == 1).all()
        # first-use order: the first piece holds what the first touching step needs
        touching = [st for st in steps if st[0] in (0, 2, 3, 5) and st[4] > 0]
        if touching:
            st = touching[0]
            assert h2d[0][0] <= st[3] < h2d[0][0] + h2d[0][1]


@pytest.mark.parametrize("algo,P", [(O.HALVING_DOUBLING, 24), (O.HALVING_DOUBLING, 32),
                                    (O.RING_CHUNKED, 15), (O.RING_CHUNKED, 11)])
@pytest.mark.parametrize("N", [0, 1, 64, 1000])
def test_plan_replay_reference_test_sizes(algo, P, N):
    """The largest context sizes of gloo/test/allreduce_test.cc:251-269
    (HD up to 32 ranks, ring_chunked up to 15), value = rank pattern."""
    ins = case_inputs(P, N, O.FLOAT32, 1, 2)
    plans = [gloo_amd.plan(NAMES[algo], r, P, N) for r in range(P)]
    got = replay_plans(plans, O.SUM, O.FLOAT32, [ins[r][0] for r in range(P)])
    for r in range(P):
        assert (got[r] == P * (P - 1) / 2).all()
    exp = O.allreduce(algo, O.SUM, O.FLOAT32, ins)
    for r in range(P):
        assert same_bits(got[r], exp[r][0])


@pytest.mark.parametrize("P", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("N", [1, 255, 1000, 4099, 65537])
@pytest.mark.parametrize("dtype,op", [(O.FLOAT32, O.SUM), (O.FLOAT16, O.SUM),
                                      (O.FLOAT32, O.MAX), (O.INT32, O.PRODUCT)])
def test_replicated_ring_chunked_is_bit_identical(P, N, dtype, op):
    ins = case_inputs(P, N, dtype, 1, 0, seed=41)
    plans = [gloo_amd.plan("ring_chunked_repl", r, P, N, with_folds=True) for r in range(P)]
    got = replay_plans(plans, op, dtype, [ins[r][0] for r in range(P)])
    exp = O.allreduce(O.RING_CHUNKED, op, dtype, ins)
    for r in range(P):
        assert same_bits(got[r], exp[r][0]), r
    # one dependent round: all sends precede every receive
    steps = plans[0][0]
    kinds = [s[0] for s in steps]
    assert kinds.index(1) > max(i for i, k in enumerate(kinds) if k == 0)


@pytest.mark.parametrize("P", [2, 3, 7, 8])
@pytest.mark.parametrize("N", [1, 1000, 4099])
@pytest.mark.parametrize("max_seg", [128, 0])
def test_replicated_fn_ring_is_bit_identical(P, N, max_seg):
    ins = [O.fill(O.FLOAT32, N, 0, seed=5, rank=r) for r in range(P)]
    plans = [gloo_amd.plan("fn_ring_repl", r, P, N, with_folds=True, max_segment_size=max_seg)
             for r in range(P)]
    got = replay_plans(plans, O.SUM, O.FLOAT32, ins)
    exp = O.allreduce_fn(O.FN_RING, O.SUM, O.FLOAT32, [[] for _ in range(P)],
                         [[x] for x in ins], max_seg)
    for r in range(P):
        assert same_bits(got[r], exp[r][0]), r


@pytest.mark.parametrize("P", list(range(1, 16)))
@pytest.mark.parametrize("N", [0, 1, 4, 100, 1000, 4099])
@pytest.mark.parametrize("dtype,op", [(O.FLOAT32, O.SUM), (O.FLOAT16, O.SUM), (O.INT32, O.MAX),
                                      (O.FLOAT32, O.PRODUCT)], ids=str)
def test_allreduce_ring_plan_replay_matches_oracle(P, N, dtype, op):
    """gloo::AllreduceRing<T>: the step program (one round of whole-buffer
    sends, then each rank's left fold r, r-1, ..., r-P+1) replayed on the
    host equals the oracle's restatement of the reference's P-1 forwarding
    rounds, rank by rank (the reference's test grid: P = 1..15)."""
    ins = case_inputs(P, N, dtype, 1, 0, seed=98)
    plans = [gloo_amd.plan("ring", r, P, N, with_folds=True) for r in range(P)]
    got = replay_plans(plans, op, dtype, [ins[r][0] for r in range(P)])
    exp = O.allreduce(O.RING, op, dtype, ins)
    for r in range(P):
        assert same_bits(got[r], exp[r][0]), "rank %d" % r


BCUBE_GRID = ([(2, P) for P in (1, 2, 3, 4, 5, 6, 8, 16)] + [(3, P) for P in (1, 2, 3, 4, 7, 9, 27)]
              + [(4, P) for P in (1, 4, 5, 8, 16)])


@pytest.mark.parametrize("base,P", BCUBE_GRID, ids=["b%d-P%d" % g for g in BCUBE_GRID])
@pytest.mark.parametrize("N", [0, 1, 3, 64, 1000, 4099])
@pytest.mark.parametrize("dtype,op", [(O.FLOAT32, O.SUM), (O.FLOAT16, O.SUM), (O.INT32, O.MAX)],
                         ids=str)
def test_allreduce_bcube_plan_replay_matches_oracle(base, P, N, dtype, op):
    """gloo::AllreduceBcube<T>: the step program (the reference's groups of
    `base` ranks, its ranges incl. the wrap-around at tiny N, peers in group
    order) replayed on the host equals the oracle's restatement, which
    equals the compiled reference on the same grid."""
    ins = case_inputs(P, N, dtype, 1, 0, seed=97)
    plans = [gloo_amd.plan("bcube:%d" % base, r, P, N, with_folds=True) for r in range(P)]
    got = replay_plans(plans, op, dtype, [ins[r][0] for r in range(P)])
    exp = O.allreduce(O.BCUBE, op, dtype, ins, base=base)
    for r in range(P):
        assert same_bits(got[r], exp[r][0]), "rank %d" % r
