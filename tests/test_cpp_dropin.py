"""The C++ drop-in surface (include/gloo_amd/gloo_amd.hpp): compiles on CPU;
the reference's allreduce test cases written against it run on the GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "dropin_test.cc")
LIBDIR = os.path.join(ROOT, "gloo_amd")


def build(out):
    cmd = ["g++", "-std=c++17", "-O2", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           "-I" + os.path.join(ROOT, "include"), SRC, "-o", out, "-L" + LIBDIR, "-lgloo_amd",
           "-L/opt/rocm/lib", "-lamdhip64", "-lpthread", "-Wl,-rpath," + LIBDIR]
    subprocess.check_call(cmd)


def test_dropin_header_compiles(tmp_path):
    build(str(tmp_path / "dropin_test"))


def test_dropin_host_function_allreduce(tmp_path):
    """gloo_amd::allreduce(opts) with a capturing lambda on host buffers
    (glx_allreduce_host_fn through the header): no GPU needed."""
    exe = str(tmp_path / "dropin_test")
    build(exe)
    p = subprocess.run([exe, "--host-fn"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "all passed" in p.stdout


@pytest.mark.gpu
def test_dropin_reference_cases_on_gpu(tmp_path):
    exe = str(tmp_path / "dropin_test")
    build(exe)
    p = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "all passed" in p.stdout


@pytest.mark.widening
def test_dropin_widening_cases_on_gpu(tmp_path):
    """The round-4 widening outside the contract (HipAllreduceRing / Bcube /
    Local): `pytest -m widening` on a GPU box."""
    exe = str(tmp_path / "dropin_test")
    build(exe)
    p = subprocess.run([exe, "--widening"], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "all passed" in p.stdout
