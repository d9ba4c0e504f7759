import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden", "xrs_golden.npz")
GOLDEN_CODECS = os.path.join(ROOT, "tests", "golden", "xrs_golden_codecs.npz")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def golden_codecs():
    with np.load(GOLDEN_CODECS, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture
def rng():
    # Fixed seeds (the reference seeds from the clock, xrs_test.go:26-31).
    return np.random.Generator(np.random.PCG64(0x5EED))
