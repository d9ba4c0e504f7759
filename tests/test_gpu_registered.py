"""GPU tests of the per-stripe calls on caller-registered host memory
(xrs_host_register / xrs_host_alloc: in place for a lone sync call, the
queue's table mode for coalesced calls).  The cases live in
tests/gpu_registered_cases.py; each test function runs there in a child
pytest process of its own, and this file asserts that it passed.

Why a child per case: over rounds 5-6, 5 full GPU-suite runs met an
illegal-address error at the first pageable PyTorch copy of the test file
that follows these cases (test_gpu_shards.py), after every case here had
passed and the device had been synchronized; keeping the unregistered
arenas alive did not prevent it, and with every kernel and copy serialized
(AMD_SERIALIZE_KERNEL=3, AMD_SERIALIZE_COPY=3) the copy itself reports it
(profiles/r06_fault_diag.log).  The cases themselves are
bit-exact in every run; a process that ran them ends here, so whatever
runtime state they leave cannot reach another test.  Reference calls:
xrs.go:103-387."""
import ast
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = os.path.join(ROOT, "tests", "gpu_registered_cases.py")


def _case_names():
    with open(CASES) as f:
        tree = ast.parse(f.read())
    return [n.name for n in tree.body if isinstance(n, ast.FunctionDef) and n.name.startswith("test_")]


@pytest.mark.parametrize("case", _case_names())
def test_registered_case_in_child(case):
    cmd = [sys.executable, "-u", "-m", "pytest", f"{CASES}::{case}", "-q", "-m", "gpu",
           "-p", "no:cacheprovider", "--timeout", "300", "--timeout-method", "thread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=ROOT,
                       env=dict(os.environ))
    out = r.stdout[-3000:] + r.stderr[-3000:]
    assert r.returncode == 0, out
    assert " passed" in r.stdout and " failed" not in r.stdout, out
