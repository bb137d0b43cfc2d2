"""CPU: the geometry the device-driven engines (xgmi_kernels.hip) run on --
glx_device_layout, exactly what HipPlanExecutor hands the one-shot and
two-shot kernels -- replayed on the host element by element the way the
kernels compute (per slice, chain folds acc = op(x[chain[k]], acc)) must
reproduce the oracle bit for bit at every P up to 8 (the GPU tests can only
run P <= 4 processes on the one-GPU boxes), and its slicing must cover every
element exactly once with whole 16-byte vectors per slice."""
import numpy as np
import pytest

import gloo_amd
from helpers import case_inputs, same_bits
from oracle import oracle as O

ESIZE = {O.FLOAT32: 4, O.FLOAT16: 2, O.INT32: 4, O.INT8: 1, O.FLOAT64: 8}


def chain_fold(op, dtype, xs, chain, lo, hi):
    """acc = x[chain[0]]; acc = op(x[chain[k]], acc) -- the ring's operand
    order (the newer rank's value is the in-place destination)."""
    acc = np.array(xs[chain[0]][lo:hi], copy=True)
    for r in chain[1:]:
        acc = O.reduce(op, dtype, np.array(xs[r][lo:hi], copy=True), acc)
    return acc


def check_slicing(lay, length, esize, max_slices):
    G, sl = lay["G"], lay["slice"]
    assert 1 <= G <= max(1, max_slices)
    assert sl % (16 // esize) == 0 and sl >= 4096 // esize
    assert G * sl >= length and (G - 1) * sl < max(length, 1)


def oneshot_replay(name, P, N, dtype, op, xs, max_slices):
    es = ESIZE[dtype]
    out = []
    for r in range(P):
        lay = gloo_amd.device_layout(name, r, P, N, es, max_slices)
        check_slicing(lay, N, es, max_slices)
        res = np.array(xs[r], copy=True)
        covered = np.zeros(N, dtype=np.int32)
        # per workgroup slice, per job: the kernel's loop structure
        for w in range(lay["G"]):
            e0, e1 = w * lay["slice"], min((w + 1) * lay["slice"], N)
            for off, ln, chain in lay["jobs"]:
                assert sorted(chain) == list(range(P))
                a, b = max(off, e0), min(off + ln, e1)
                if a < b:
                    res[a:b] = chain_fold(op, dtype, xs, chain, a, b)
                    covered[a:b] += 1
        assert (covered == 1).all(), "rank %d: elements folded %s times" % (
            r, sorted(set(covered.tolist())))
        out.append(res)
    return out


def twoshot_replay(name, P, N, dtype, op, xs, max_slices):
    es = ESIZE[dtype]
    lays = [gloo_amd.device_layout(name, r, P, N, es, max_slices) for r in range(P)]
    # every rank sees the same ranges and slicing; non-empty ranges tile [0, N)
    for lay in lays[1:]:
        assert lay["ranges"] == lays[0]["ranges"]
        assert (lay["G"], lay["slice"]) == (lays[0]["G"], lays[0]["slice"])
    ranges = lays[0]["ranges"]
    spans = sorted((o, n) for o, n in ranges if n > 0)
    at = 0
    for o, n in spans:
        assert o == at
        at += n
    assert at == N
    max_len = max(n for _, n in ranges)
    assert lays[0]["max_len"] == max_len
    check_slicing(lays[0], max_len, es, max_slices)
    # phase 2: owner j folds slice w of its range along its chain; phase 3:
    # every rank takes every owner's finished slices
    finished = {}
    for j in range(P):
        off, ln = ranges[j]
        if ln == 0:
            continue
        assert sorted(lays[j]["my_chain"]) == list(range(P))
        parts = []
        for w in range(lays[j]["G"]):
            a = off + min(w * lays[j]["slice"], ln)
            b = off + min((w + 1) * lays[j]["slice"], ln)
            if a < b:
                parts.append(chain_fold(op, dtype, xs, lays[j]["my_chain"], a, b))
        finished[j] = np.concatenate(parts)
        assert finished[j].size == ln
    out = []
    for r in range(P):
        res = np.array(xs[r], copy=True)
        for j, v in finished.items():
            off, ln = ranges[j]
            res[off:off + ln] = v
        out.append(res)
    return out


CLASS_CASES = [(P, N) for P in range(2, 9) for N in (1, 3, 255, 256, 257, 1000, 4099, 65539)]


@pytest.mark.parametrize("P,N", CLASS_CASES)
@pytest.mark.parametrize("engine", ["oneshot", "twoshot"])
def test_device_layout_replay_ring_chunked(P, N, engine):
    ins = case_inputs(P, N, O.FLOAT32, 1, 0, seed=71)
    xs = [ins[r][0] for r in range(P)]
    exp = O.allreduce(O.RING_CHUNKED, O.SUM, O.FLOAT32, ins)
    if engine == "oneshot":
        got = oneshot_replay("ring_chunked_repl", P, N, O.FLOAT32, O.SUM, xs, 256)
    else:
        got = twoshot_replay("ring_chunked_mesh", P, N, O.FLOAT32, O.SUM, xs, 256)
    for r in range(P):
        assert same_bits(got[r], exp[r][0]), "rank %d" % r


@pytest.mark.parametrize("dtype,op", [(O.FLOAT16, O.SUM), (O.FLOAT16, O.MAX),
                                      (O.INT32, O.PRODUCT), (O.INT8, O.SUM),
                                      (O.FLOAT64, O.MIN)])
@pytest.mark.parametrize("engine", ["oneshot", "twoshot"])
@pytest.mark.parametrize("max_slices", [256, 3, 1])
def test_device_layout_replay_dtypes_and_small_grids(dtype, op, engine, max_slices):
    """Grids capped below the natural slice count (a GPU shared by several
    ranks) still cover every element once."""
    P, N = 8, 70001
    ins = case_inputs(P, N, dtype, 1, 0, seed=72)
    xs = [ins[r][0] for r in range(P)]
    exp = O.allreduce(O.RING_CHUNKED, op, dtype, ins)
    fn = oneshot_replay if engine == "oneshot" else twoshot_replay
    name = "ring_chunked_repl" if engine == "oneshot" else "ring_chunked_mesh"
    got = fn(name, P, N, dtype, op, xs, max_slices)
    for r in range(P):
        assert same_bits(got[r], exp[r][0]), "rank %d" % r


@pytest.mark.parametrize("P", [2, 3, 5, 8])
@pytest.mark.parametrize("N", [1, 1000, 65536, 262147])
@pytest.mark.parametrize("engine", ["oneshot", "twoshot"])
def test_device_layout_replay_fn_ring(P, N, engine):
    """gloo::allreduce(opts) RING's result (UNSPECIFIED / RING_MESH) on the
    device engines: chains start one rank left of the owner (allreduce.cc)."""
    data = case_inputs(P, N, O.FLOAT32, 1, 0, seed=73)
    xs = [data[r][0] for r in range(P)]
    exp = O.allreduce_fn(O.FN_RING, O.SUM, O.FLOAT32, [[] for _ in range(P)], data)
    fn = oneshot_replay if engine == "oneshot" else twoshot_replay
    name = "fn_ring_repl" if engine == "oneshot" else "fn_ring_mesh"
    got = fn(name, P, N, O.FLOAT32, O.SUM, xs, 256)
    for r in range(P):
        assert same_bits(got[r], exp[r][0]), "rank %d" % r


def test_device_layout_rejects_other_schedules():
    with pytest.raises(gloo_amd.EnforceNotMet):
        gloo_amd.device_layout("ring_chunked", 0, 4, 1000)
    with pytest.raises(gloo_amd.EnforceNotMet):
        gloo_amd.device_layout("ring_chunked_mesh", 0, 9, 1000)  # P > 8
