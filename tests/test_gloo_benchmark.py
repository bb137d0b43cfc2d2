"""tools/gloo_benchmark.py -- the reference benchmark runner's command line,
inputs, verification and table (gloo/benchmark/{main,cuda_main,runner}.cc)
on gloo_amd.  CPU: the input / expectation / check helpers against a numpy
allreduce of the same inputs.  GPU: real runs, one process per rank."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gloo_benchmark as gb  # noqa: E402


@pytest.mark.parametrize("P,inputs,n", [(1, 1, 100), (2, 1, 1000), (3, 2, 500), (8, 1, 5000)])
@pytest.mark.parametrize("dtype", [np.float32, np.float16])
def test_expected_values_are_the_allreduce_of_the_inputs(P, inputs, n, dtype):
    ins = [gb.inputs_for(np, dtype, P, r, inputs, n) for r in range(P)]
    # the allreduce of every rank's every input, summed in float64 (exact)
    total = sum(x.astype(np.float64) for per in ins for x in per)
    exp64, exp = gb.expected_for(np, dtype, "cuda_allreduce_ring_chunked", P, 0, inputs, n)
    if dtype == np.float32:
        np.testing.assert_array_equal(total, exp64)
    with np.errstate(over="ignore"):
        got = total.astype(dtype)
    assert gb.check(np, dtype, got, exp64, exp, P * inputs).size == 0


@pytest.mark.parametrize("P,inputs", [(1, 1), (2, 3), (4, 2)])
def test_local_expectation_is_this_ranks_inputs_only(P, inputs):
    n = 777
    for r in range(P):
        ins = gb.inputs_for(np, np.float32, P, r, inputs, n)
        local = sum(x.astype(np.float64) for x in ins)
        exp64, exp = gb.expected_for(np, np.float32, "allreduce_local", P, r, inputs, n)
        np.testing.assert_array_equal(local, exp64)
        if inputs == 1:  # the reference's own expectation (main.cc:268-283)
            np.testing.assert_array_equal(exp64, np.arange(n) * P + r)


def test_check_is_exact_in_range_and_allows_rounding_beyond():
    n = 10
    exp64 = np.arange(n, dtype=np.float64) * 3 + 1
    exp = exp64.astype(np.float32)
    got = exp.copy()
    got[4] += 1  # an integer off by one where the type is exact: reported
    assert list(gb.check(np, np.float32, got, exp64, exp, 2)) == [4]
    big64 = np.array([2.0 ** 25 + 1, 2.0 ** 26 + 3])
    big = big64.astype(np.float32)
    near = (big64 * (1 + 1e-7)).astype(np.float32)
    assert gb.check(np, np.float32, near, big64, big, 2).size == 0
    far = (big64 * 1.01).astype(np.float32)
    assert gb.check(np, np.float32, far, big64, big, 2).size == 2


def test_float16_outputs_the_reference_keeps_stale_are_not_flagged():
    """gloo's float16 sum of 14744 + 14744 is 14744 (its operator= skips the
    store, gloo/types.h:129-134; the compiled reference's AllreduceRing gives
    exactly that at index 7371 of the benchmark inputs, P = 2): the check
    leaves fp16 values >= 15360 alone, and still flags smaller ones."""
    exp64 = np.array([29488.0, 1000.0])
    exp = exp64.astype(np.float16)
    got = np.array([14744.0, 1000.0], dtype=np.float16)
    assert gb.check(np, np.float16, got, exp64, exp, 2).size == 0
    got[1] = 999.0
    assert list(gb.check(np, np.float16, got, exp64, exp, 2)) == [1]


def test_float16_overflow_to_inf_matches_inf():
    exp64 = np.array([70000.0, 1.0])
    with np.errstate(over="ignore"):
        exp = exp64.astype(np.float16)
    got = np.array([np.inf, 1.0], dtype=np.float16)
    assert gb.check(np, np.float16, got, exp64, exp, 2).size == 0


def test_command_line_mirrors_the_reference():
    a = gb.parse_args(["-s", "2", "-r", "1", "--shared-path", "/tmp/x", "--elements", "100",
                       "--inputs", "2", "--iteration-time", "500ms", "--no-verify",
                       "--halfprecision", "--base", "3", "cuda_allreduce_halving_doubling"])
    assert (a.size, a.rank, a.elements, a.inputs, a.verify, a.halfprecision, a.base) == \
        (2, 1, 100, 2, False, True, 3)
    assert a.iteration_time == 500 * 10**6
    assert gb.parse_time("2s") == 2 * 10**9 and gb.parse_time("100us") == 100000
    with pytest.raises(SystemExit):
        gb.parse_args(["-s", "2", "-r", "0", "allreduce_ring"])  # no rendezvous path
    # every class algorithm of the reference's allreduce benchmarks
    for name in ("allreduce_ring", "allreduce_ring_chunked", "allreduce_halving_doubling",
                 "allreduce_bcube", "allreduce_local", "cuda_allreduce_ring",
                 "cuda_allreduce_ring_chunked", "cuda_allreduce_halving_doubling",
                 "cuda_allreduce_halving_doubling_pipelined", "cuda_allreduce_bcube",
                 "cuda_allreduce_local"):
        assert gb.parse_args([name]).benchmark == name


def _run(tmp_path, P, args, timeout=150):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    if P > 1:
        env["GPU_MAX_HW_QUEUES"] = "1"
    procs = [subprocess.Popen(
        [sys.executable, os.path.join(ROOT, "tools", "gloo_benchmark.py"), "-s", str(P),
         "-r", str(r), "--shared-path", str(tmp_path)] + args,
        stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, cwd=ROOT) for r in range(P)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode(errors="replace"))
    return [p.returncode for p in procs], outs


# the reference benchmark's command line is outside the SURVEY 8 contract
# (DESIGN.md 8): its GPU runs carry the `widening` marker, not `gpu`
@pytest.mark.widening
@pytest.mark.parametrize("bench,P,extra", [
    ("cuda_allreduce_ring_chunked", 2, ["--inputs", "2"]),
    ("cuda_allreduce_halving_doubling_pipelined", 3, []),
    ("cuda_allreduce_ring", 2, ["--halfprecision"]),
    ("cuda_allreduce_bcube", 4, []),
    ("allreduce_local", 2, ["--inputs", "3"]),
])
def test_benchmark_runs_and_verifies(tmp_path, bench, P, extra):
    rcs, outs = _run(tmp_path, P, ["--elements", "100000", "--iteration-count", "5", "--json",
                                   bench] + extra)
    assert rcs == [0] * P, outs
    assert "Mismatch" not in "".join(outs)
    lines = [l for l in outs[0].splitlines() if l.startswith("{")]
    assert len(lines) == 1
    import json
    rec = json.loads(lines[0])
    assert rec["elements"] == 100000 and rec["iterations"] == 5 and rec["verified"]
    assert "BENCHMARK RESULTS" in outs[0] and bench.upper() in outs[0]


@pytest.mark.widening
def test_benchmark_sweep_with_iteration_time(tmp_path):
    rcs, outs = _run(tmp_path, 2, ["--iteration-time", "20ms", "--json",
                                   "cuda_allreduce_ring_chunked"])
    assert rcs == [0, 0], outs
    recs = [l for l in outs[0].splitlines() if l.startswith("{")]
    assert len(recs) == 15  # 100, 200, 500 ... 5M elements (runner.cc:256-266)
