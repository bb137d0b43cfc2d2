"""Positive controls for the suite's stale-data checks.

The device engines hand data over through flag words with the narrow sync
(xgmi_kernels.hip release_stores / acquire_loads).  A check that
cannot fail a deliberately broken hand-off certifies nothing, so the library
carries TEST-ONLY broken sync modes (kernels.h kSyncNoAcquire ..
kSyncCachedSlots, GLOO_AMD_SYNC=unsafe_*) and these tests show which of them
the checks catch on one GPU:

* the soak at a small buffer (4096 elements: every workgroup re-reads a few KB
  of landing slot its CU read two messages before within the same launch --
  L1-warm, the guide's near-certain stale case) is exact under the product's
  narrow sync at P = 4 and 8, and wrong in (nearly) every run of the ring on
  every rank once the consumer's acquire is dropped (unsafe_noacquire;
  profiles/round6/sync_control_*.json: 200 of 200 runs at P = 4 and 8);
* dropping the producer's store-completion wait and the workgroup barrier
  before the flag (unsafe_norelease) is NOT caught at 4096 or 65,536
  elements -- a workgroup's slice is then one wave's, and it lands before any
  consumer's poll -- but IS caught at 1 M elements, where a slice spans every
  wave of the workgroup and the flag can overtake the other waves' stores:
  the two-shot mesh wrong in 91-100 of 100 runs on every rank at P = 4 and 8
  (the plan kernel's ring and halving-doubling in 0-2; 16 M elements: the
  mesh in 25-46; profiles/round6/sync_control_release_1M_16M.json);
* at the north-star size (2^26 elements per rank) the plan kernel's own ring
  -- the north star's engine -- is wrong in 29-30 of 30 runs on every rank
  without the release, and exact with it (profiles/round6/
  sync_control_release_64M_plan_kernel.json).
"""
import os
import re
import subprocess
import sys
import tempfile

import pytest

from helpers import rank_env

WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mp_worker.py")
SMALL = 4096
LARGE = 1 << 20
NORTH_STAR = 1 << 26  # 256 MiB fp32 per rank


def small_soak(P, runs, sync, n=SMALL):
    env = rank_env(P)
    env["GLOO_AMD_SYNC"] = sync
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, WORKER, d, str(r), str(P),
                                   "soak:%d:delays:%d" % (runs, n)],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(P)]
        outs = []
        for p in procs:
            try:
                o, _ = p.communicate(timeout=150)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs.append(o.decode(errors="replace"))
    bad = []
    for o in outs:
        m = re.search(r"BADRUNS rank \d+ (\{.*?\}) of", o)
        assert m, o[-2000:]
        bad.append(eval(m.group(1)))  # noqa: S307 - the worker's own dict literal
    eng = [line for line in outs[0].splitlines() if line.startswith("ENGINES")][0]
    return [p.returncode for p in procs], bad, eng, outs


@pytest.mark.gpu
@pytest.mark.parametrize("P", [4, 8])
def test_small_buffer_soak_exact_under_the_product_sync(P):
    """The sharp detector on the product: L1-warm re-reads of landing slots
    within one launch, 200 runs of every engine, every run exact."""
    rcs, bad, eng, outs = small_soak(P, 200, "narrow")
    assert "'ring': 'devsteps'" in eng, eng
    assert rcs == [0] * P and all(b == {} for b in bad), (rcs, bad, outs[0][-2000:])


@pytest.mark.gpu
@pytest.mark.parametrize("P", [4, 8])
def test_small_buffer_soak_catches_a_missing_acquire(P):
    """Positive control: with the consumer's acquire dropped (test-only
    kSyncNoAcquire) the same soak fails -- the plan kernel's ring reads stale
    L1 lines of its landing slot; measured 200 of 200 runs on every rank."""
    runs = 100
    rcs, bad, eng, _ = small_soak(P, runs, "unsafe_noacquire")
    assert "'ring': 'devsteps'" in eng, eng
    assert all(rc != 0 for rc in rcs), rcs
    for r, b in enumerate(bad):
        assert b.get("ring", 0) >= runs // 2, (r, b)


@pytest.mark.gpu
@pytest.mark.parametrize("P", [4, 8])
def test_large_buffer_soak_exact_under_the_product_sync(P):
    """The release-side detector on the product: 1 M elements, every
    workgroup's slice spread over all its waves, 100 runs of every engine,
    every run exact."""
    rcs, bad, eng, outs = small_soak(P, 100, "narrow", LARGE)
    assert "'mesh': 'twoshot'" in eng, eng
    assert rcs == [0] * P and all(b == {} for b in bad), (rcs, bad, outs[0][-2000:])


@pytest.mark.gpu
@pytest.mark.parametrize("P", [4, 8])
def test_large_buffer_soak_catches_a_missing_release(P):
    """Positive control for the producer side: with every wave's store wait
    and the barrier before the flag dropped (test-only kSyncNoRelease) the
    two-shot mesh hands over data still in flight; measured wrong in 91-100
    of 100 runs on every rank."""
    runs = 40
    rcs, bad, eng, _ = small_soak(P, runs, "unsafe_norelease", LARGE)
    assert "'mesh': 'twoshot'" in eng, eng
    assert all(rc != 0 for rc in rcs), rcs
    for r, b in enumerate(bad):
        assert b.get("mesh", 0) >= runs // 2, (r, b)


@pytest.mark.gpu
def test_north_star_size_plan_kernel_exact_and_catches_a_missing_release():
    """At the north star's 256 MiB per rank, P = 4: the plan kernel's ring
    (mp_worker.py soak "ring_dev") exact under the product sync, and wrong in
    (nearly) every run on every rank once the release is dropped."""
    runs = 6
    rcs, bad, eng, outs = small_soak(4, runs, "narrow", NORTH_STAR)
    assert "'ring_dev': 'devsteps'" in eng, eng
    assert rcs == [0] * 4 and all(b == {} for b in bad), (rcs, bad, outs[0][-2000:])
    rcs, bad, eng, _ = small_soak(4, runs, "unsafe_norelease", NORTH_STAR)
    assert all(rc != 0 for rc in rcs), rcs
    for r, b in enumerate(bad):
        assert b.get("ring_dev", 0) >= runs // 2, (r, b)
