"""CPU: randomized shapes for the product's step programs (hypothesis, fixed
seed, bounded example counts).  The parametrized tests pin the reference
suites' grids; these draw rank counts, element counts, element sizes,
segment sizes and workgroup counts off those grids, where chunk boundaries,
16-byte phases and empty chunks fall differently:

* every schedule's compiled programs (glx_plan -- what the executor runs),
  replayed with the landing / credit rules, equal the oracle bit for bit;
* the plan kernel's protocol simulated per (rank, workgroup) with drifting
  workgroups (test_plan_kernel_sim.simulate) finishes without a stall or a
  clobbered landing region and equals the oracle, for every program
  glx_plan_sync calls safe."""
import pytest

hyp = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, seed, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

import gloo_amd  # noqa: E402
from gloo_amd import algorithms as A  # noqa: E402
from helpers import case_inputs, replay_plans, same_bits  # noqa: E402
from oracle import oracle as O  # noqa: E402
from test_plan_kernel_sim import expected, simulate  # noqa: E402

SETTINGS = dict(max_examples=300, deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.too_slow])
CLASS = {"ring_chunked": O.RING_CHUNKED, "halving_doubling": O.HALVING_DOUBLING,
         "ring_chunked_mesh": O.RING_CHUNKED}
DTYPES = {O.FLOAT32: 4, O.FLOAT16: 2, O.FLOAT64: 8, O.INT32: 4}


@settings(**SETTINGS)
@seed(20261017)
@given(name=st.sampled_from(sorted(CLASS)), P=st.integers(1, 17),
       N=st.one_of(st.integers(0, 70), st.integers(71, 200000)),
       dtype=st.sampled_from(sorted(DTYPES)), op=st.sampled_from([O.SUM, O.MAX, O.PRODUCT]))
def test_class_plans_replay_matches_oracle(name, P, N, dtype, op):
    ins = case_inputs(P, N, dtype, 1, 0, seed=P * 1000 + N % 997)
    plans = [gloo_amd.plan(name, r, P, N, with_folds=True, esize=DTYPES[dtype])
             for r in range(P)]
    got = replay_plans(plans, op, dtype, [ins[r][0] for r in range(P)])
    exp = O.allreduce(CLASS[name], op, dtype, ins)
    for r in range(P):
        assert same_bits(got[r], exp[r][0]), "rank %d" % r


@settings(**SETTINGS)
@seed(20261018)
@given(algo=st.sampled_from(["fn_ring", "fn_ring_mesh", "fn_bcube"]), P=st.integers(1, 12),
       N=st.integers(1, 60000), dtype=st.sampled_from([O.FLOAT32, O.FLOAT16]),
       max_seg=st.sampled_from([0, 16, 128, 1000, 4096, 1 << 16]),
       piece=st.sampled_from([0, 4, 64, 4096]))
def test_fn_plans_replay_matches_oracle(algo, P, N, dtype, max_seg, piece):
    code = {"fn_ring": O.FN_RING, "fn_ring_mesh": O.FN_RING, "fn_bcube": O.FN_BCUBE}[algo]
    es = DTYPES[dtype]
    data = [O.fill(dtype, N, 0, seed=7, rank=r) for r in range(P)]
    plans = [A.plan(algo, r, P, N, with_folds=True, esize=es, max_segment_size=max_seg,
                    min_piece_bytes=piece) for r in range(P)]
    got = replay_plans(plans, O.SUM, dtype, data)
    exp = O.allreduce_fn(code, O.SUM, dtype, [[] for _ in range(P)], [[x] for x in data],
                         max_seg)
    for r in range(P):
        assert same_bits(got[r], exp[r][0]), "rank %d" % r


@settings(**dict(SETTINGS, max_examples=200))
@seed(20261019)
@given(name=st.sampled_from(["ring_chunked", "halving_doubling", "fn_ring", "fn_bcube",
                             "ring_chunked_mesh"]),
       P=st.integers(2, 8), N=st.integers(1, 40000), G=st.integers(1, 9),
       fuse=st.booleans())
def test_plan_kernel_protocol_random_shapes(name, P, N, G, fuse):
    if not all(gloo_amd.plan_sync(name, r, P, N, G)["safe"] for r in range(P)):
        return  # the executor keeps host-issued steps for this program
    ins = case_inputs(P, N, O.FLOAT32, 1, 0, seed=N % 101)
    got = simulate(name, P, N, G, O.SUM, ins, fuse=fuse)
    exp = expected(name, P, O.SUM, ins, 2)
    for r in range(P):
        assert same_bits(got[r], exp[r][0]), "rank %d" % r
