"""GPU tests of the one-process multi-GPU group (xrs_group_*): a host-resident
batch split across members, against the oracle.  The box has one GPU, so the
members are the same device listed more than once: the split, the threads and
the per-member codecs are exercised; cross-device PCIe scaling is not."""
import ctypes

import numpy as np
import pytest

import xrs_amd
from oracle.oracle_c import OracleXRS

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
D, P = 12, 4


def _pinned(nbytes):
    p = xrs_amd.lib().xrs_host_alloc(nbytes)
    assert p
    return p, np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
@pytest.mark.parametrize("pinned", [True, False])
@pytest.mark.parametrize("size,n", [(4096, 1001), (1 << 20, 7), (1026, 5)])
def test_group_host_vs_oracle(rng, devices, pinned, size, n):
    stripe = 16 * size
    if pinned:
        ptr, buf = _pinned(n * stripe)
    else:
        buf = np.empty(n * stripe, np.uint8)
        ptr = buf.ctypes.data
    buf[:] = rng.integers(0, 256, size=n * stripe, dtype=np.uint8)
    ref = buf.reshape(n, 16, size).copy()
    OracleXRS(D, P).encode_batch(ref, size, n)
    g = xrs_amd.XRSGroup(D, P, devices)
    assert len(g) == len(devices)
    g.encode_host(ptr, size, size, stripe, n)
    v = buf.reshape(n, 16, size)
    assert np.array_equal(v, ref)
    k = 4
    v[:, k] = 0
    g.reconst_one_host(ptr, size, size, stripe, n, k)
    assert np.array_equal(v, ref)
    # general Reconst (one data + one piggybacked parity lost), side effects
    # included: the stripes match the oracle's per-stripe Reconst
    lost = [2, 14]
    has = [j for j in range(D + P) if j not in lost]
    v[:, lost] = 0xA5
    exp = v.copy()
    o = OracleXRS(D, P)
    for s in range(n):
        w = [exp[s, i].copy() for i in range(D + P)]
        o.reconst(w, has, lost)
        exp[s] = np.stack(w)
    g.reconst_host(ptr, size, size, stripe, n, has, lost)
    assert np.array_equal(v, exp)
    # Update (row 6 <- new data) and Replace(rows 1, 10) with data in a
    # separate buffer, parity in place
    v[:] = ref
    new = rng.integers(0, 256, size=(n, size), dtype=np.uint8)
    rows = [1, 10]
    data = rng.integers(0, 256, size=(n, 2, size), dtype=np.uint8)
    exp = ref.copy()
    for s in range(n):
        par = [exp[s, D + r] for r in range(P)]
        o.update(exp[s, 6].copy(), new[s], 6, par)
        o.replace([data[s, 0], data[s, 1]], rows, par)
    g.update_host(ptr + 6 * size, stripe, new.ctypes.data, size, size, 6, ptr + D * size, size,
                  stripe, n)
    g.replace_host(data.ctypes.data, size, 2 * size, rows, size, ptr + D * size, size, stripe, n)
    assert np.array_equal(v, exp)
    del g
    if pinned:
        xrs_amd.lib().xrs_host_free(ptr)


def test_group_errors():
    with pytest.raises(xrs_amd.XRSError, match="invalid argument"):
        xrs_amd.XRSGroup(D, P, [])
    with pytest.raises(xrs_amd.XRSError, match="invalid argument"):
        xrs_amd.XRSGroup(D, P, [torch.cuda.device_count()])
    with pytest.raises(xrs_amd.XRSError, match="illegal parity"):
        xrs_amd.XRSGroup(D, 1, [0])
    g = xrs_amd.XRSGroup(D, P, [0, 0])
    buf = np.zeros(16 * 64, np.uint8)
    with pytest.raises(xrs_amd.XRSError, match="^illegal data index: 12$"):
        g.reconst_one_host(buf.ctypes.data, 64, 64, 16 * 64, 1, 12)
    with pytest.raises(xrs_amd.XRSError, match="^vect size not even: 63$"):
        g.encode_host(buf.ctypes.data, 63, 64, 16 * 64, 1)


def test_group_replace_error_order_matches_codec():
    """Too many rows and an odd size: the group and the single codec both
    report the size first (check_replace order, as the oracle)."""
    g = xrs_amd.XRSGroup(D, P, [0, 0])
    x = xrs_amd.XRS(D, P)
    data = np.zeros(64, np.uint8)
    par = np.zeros(16 * 64, np.uint8)
    rows = list(range(D + 1))
    for call in (lambda: g.replace_host(data.ctypes.data, 0, 0, rows, 63, par.ctypes.data, 64,
                                        4 * 64, 1),
                 lambda: x.replace_host(data.ctypes.data, 0, 0, rows, 63, par.ctypes.data, 64,
                                        4 * 64, 1)):
        with pytest.raises(xrs_amd.XRSError, match="^vect size not even: 63$"):
            call()
    for call in (lambda: g.replace_host(data.ctypes.data, 0, 0, rows, 64, par.ctypes.data, 64,
                                        4 * 64, 1),
                 lambda: x.replace_host(data.ctypes.data, 0, 0, rows, 64, par.ctypes.data, 64,
                                        4 * 64, 1)):
        with pytest.raises(xrs_amd.XRSError, match="^illegal vects$"):
            call()
