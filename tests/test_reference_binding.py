"""The reference-side drop-in: integration/gloo/hip_allreduce.h (the header a
gloo maintainer adds next to gloo/cuda_allreduce_ring_chunked.h) compiled
against the REFERENCE's own headers and linked with its objects (its
Context, rendezvous stores, tcp transport, CPU algorithms) plus
libgloo_amd.so -- `make -C oracle binding` -> oracle/_ref/binding_test
(tests/cpp/binding_test.cc).  The product library itself never links
reference code.

CPU: built here (where /root/reference exists) and run without a GPU: type
and ReductionFunction::type() mapping, CUSTOM refused with
gloo::EnforceNotMet, glx errors as gloo::IoException / EnforceNotMet, the
rendezvous::Store bridge.  GPU: the prebuilt binary (it travels with the
tree; the box has no /root/reference) runs P thread-ranks bootstrapped the
reference's way and compares HipAllreduceRingChunked / HalvingDoubling bit
for bit with the reference's own CPU algorithms in the same process."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "binding_test")
REF = "/root/reference/gloo"


def ensure_built():
    if os.path.isdir(REF):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "binding"])
    if not os.path.exists(BIN):
        pytest.skip("oracle/_ref/binding_test not built (needs /root/reference)")


def test_binding_compiles_against_reference_and_runs_cpu():
    ensure_built()
    p = subprocess.run([BIN, "cpu"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "binding_test cpu: OK" in p.stdout


@pytest.mark.gpu
def test_binding_vs_reference_cpu_algorithms_on_gpu():
    if not os.path.exists(BIN):
        pytest.skip("oracle/_ref/binding_test was not built in the build container")
    # below the GPU box's 180 s silence limit: a hang fails the test instead
    p = subprocess.run([BIN, "gpu"], capture_output=True, text=True, timeout=150)
    print(p.stdout)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "binding_test gpu: OK" in p.stdout
