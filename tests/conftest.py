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


@pytest.fixture(autouse=True)
def _device_clean_after_gpu_test(request):
    """After every GPU test, collect garbage (codecs and queues freed here, not
    inside the next test) and synchronize the device, so an asynchronous
    fault fails the test that caused it rather than a later one."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_available() or not torch.cuda.is_initialized():
        return
    import gc

    gc.collect()
    torch.cuda.synchronize()
    if os.environ.get("XRS_TEST_H2D_PROBE") == "1":  # diagnostics: a pageable copy up and back
        h = np.arange(1 << 20, dtype=np.uint32).view(np.uint8)
        assert np.array_equal(torch.from_numpy(h).cuda().cpu().numpy(), h)
        torch.cuda.synchronize()
