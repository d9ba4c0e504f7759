"""Runs the C++ port of the reference's tests (tests/cpp/xrs_test.cpp, over
include/xrs.hpp): host-logic tests on CPU, all tests on the GPU box."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "xrs_test")


def build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True)


def test_cpp_host_logic():
    build()
    r = subprocess.run([BIN, "--cpu"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout


@pytest.mark.parametrize("san", ["tsan", "asan"])
def test_hostreg_table_under_sanitizers(san):
    """The registered-range table (xrs_amd/csrc/hostreg.cpp) alone: lookups,
    readers racing register / unregister (4,000 replacements: the sanitizers'
    instrumented atomics make each grace period ~25x slower than the
    uninstrumented 0.1 ms), every replaced table freed by its writer."""
    build()
    r = subprocess.run([os.path.join(ROOT, "tests", "cpp", "build", f"hostreg_test_{san}"), "4000"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS hostreg" in r.stdout


@pytest.mark.gpu
def test_cpp_all_on_gpu():
    if not os.path.exists(BIN):
        build()
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout
