"""GPU tests of the host-resident pipelined path (xrs_encode_host,
xrs_reconst_one_host): shards start and end in host memory."""
import ctypes

import numpy as np
import pytest

import xrs_amd
from oracle.oracle_c import OracleXRS

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

D, P = 12, 4


def pinned(nbytes):
    lib = xrs_amd.lib()
    p = lib.xrs_host_alloc(nbytes)
    assert p
    arr = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))
    return p, arr


@pytest.mark.parametrize("size,n", [(4096, 5000), (1 << 20, 70), (1026, 333), (8 << 20, 9)])
@pytest.mark.parametrize("mode", ["pinned_zero_copy", "pinned_dma", "pageable"])
def test_encode_host_vs_oracle(rng, monkeypatch, size, n, mode):
    """Pinned memory runs the kernels in place over PCIe (zero copy) unless
    XRS_HOST_ZC=0 selects the copy pipeline; pageable memory always copies."""
    pin = mode != "pageable"
    if mode == "pinned_dma":
        monkeypatch.setenv("XRS_HOST_ZC", "0")
    stripe = 16 * size
    if pin:
        ptr, buf = pinned(n * stripe)
    else:
        buf = np.empty(n * stripe, np.uint8)
        ptr = buf.ctypes.data
    buf[:] = rng.integers(0, 256, size=n * stripe, dtype=np.uint8)
    ref = buf.reshape(n, 16, size).copy()
    OracleXRS(D, P).encode_batch(ref, size, n)
    x = xrs_amd.XRS(D, P)
    x.encode_host(ptr, size, size, stripe, n)
    assert np.array_equal(buf.reshape(n, 16, size), ref)
    # ReconstOne from host: erase row k everywhere, rebuild, compare
    for k in (0, 7):
        v = buf.reshape(n, 16, size)
        v[:, k] = 0
        # garbage outside the need set must not matter
        a_need, b_need = x.get_need_vects(k)
        for j in range(16):
            if j not in a_need and j != k:
                v[:, j, : size // 2] = 0xEE
        x.reconst_one_host(ptr, size, size, stripe, n, k)
        assert np.array_equal(v[:, k], ref[:, k]), k
        v[:] = ref
    if pin:
        xrs_amd.lib().xrs_host_free(ptr)


def test_encode_host_padded_layout(rng):
    size, n = 4096, 1500
    shard, stripe = size + 48, 16 * (size + 48) + 32
    buf = rng.integers(0, 256, size=n * stripe, dtype=np.uint8)
    orig = buf.copy()
    x = xrs_amd.XRS(D, P)
    x.encode_host(buf.ctypes.data, size, shard, stripe, n)
    o = OracleXRS(D, P)
    for s in (0, 1, 777, n - 1):
        v = [orig[s * stripe + i * shard:][:size].copy() for i in range(16)]
        o.encode(v)
        for i in range(16):
            off = s * stripe + i * shard
            assert np.array_equal(buf[off:off + size], v[i])
    mask = np.ones(len(buf), bool)
    for i in range(12, 16):
        for s in range(n):
            mask[s * stripe + i * shard:s * stripe + i * shard + size] = False
    assert np.array_equal(buf[mask], orig[mask])  # only parity bytes written


def test_host_zero_copy_inside_allocation(rng):
    """A batch that starts inside a pinned allocation, with a padded layout:
    the in-place path addresses it through the mapped device pointer."""
    size, n = 4096, 700
    shard, stripe = size + 64, 16 * (size + 64) + 128
    ptr, buf = pinned(n * stripe + 8192)
    off = 4096
    buf[:] = rng.integers(0, 256, size=len(buf), dtype=np.uint8)
    orig = buf.copy()
    x = xrs_amd.XRS(D, P)
    x.encode_host(ptr + off, size, shard, stripe, n)
    o = OracleXRS(D, P)
    for s in (0, 1, 345, n - 1):
        v = [orig[off + s * stripe + i * shard:][:size].copy() for i in range(16)]
        o.encode(v)
        for i in range(16):
            a = off + s * stripe + i * shard
            assert np.array_equal(buf[a:a + size], v[i]), (s, i)
    assert xrs_amd.lib().xrs_host_device_pointer(ptr)
    xrs_amd.lib().xrs_host_free(ptr)


@pytest.mark.parametrize("size,n", [(4096, 3000), (1026, 257), (1 << 20, 9)])
@pytest.mark.parametrize("mode", ["pinned_zero_copy", "pinned_dma", "pageable"])
def test_reconst_host_vs_oracle(rng, monkeypatch, size, n, mode):
    """xrs_reconst_host on a host-resident batch: clean loss patterns (only
    survivors up, written halves back) and unclean ones (repeated index, need
    inside dpHas: whole stripes both ways), side effects included."""
    pin = mode != "pageable"
    if mode == "pinned_dma":
        monkeypatch.setenv("XRS_HOST_ZC", "0")
    stripe = 16 * size
    if pin:
        ptr, buf = pinned(n * stripe)
    else:
        buf = np.empty(n * stripe, np.uint8)
        ptr = buf.ctypes.data
    o = OracleXRS(D, P)
    x = xrs_amd.XRS(D, P)
    cases = [([0, 5], [0, 5]), ([2, 13, 15], [2, 13]), ([1, 6, 9, 12], [1, 6, 9, 12]),
             ([3], [3, 3]), ([4, 7], [4, 8])]
    for lost, need in cases:
        buf[:] = rng.integers(0, 256, size=n * stripe, dtype=np.uint8)
        v = buf.reshape(n, 16, size)
        o.encode_batch(v, size, n)
        for j in lost:
            v[:, j] = 0x5A
        ref = v.copy()
        has = [j for j in range(D + P) if j not in lost]
        x.reconst_host(ptr, size, size, stripe, n, has, need)
        for s in range(0, n, max(1, n // 40)):  # a sample of stripes against the oracle
            w = [ref[s, i].copy() for i in range(D + P)]
            o.reconst(w, has, need)
            assert np.array_equal(v[s], np.stack(w)), (lost, need, s)
    if pin:
        xrs_amd.lib().xrs_host_free(ptr)


@pytest.mark.parametrize("size,n", [(4096, 2000), (1026, 100), (1 << 20, 6)])
@pytest.mark.parametrize("mode", ["pinned_zero_copy", "pinned_dma", "pageable"])
def test_update_replace_host_vs_oracle(rng, monkeypatch, size, n, mode):
    """xrs_update_host / xrs_replace_host: old, new, data and parity in
    separate host buffers (pinned in place, pinned copy pipeline, pageable);
    parity equals the oracle's per-stripe Update / Replace."""
    pin = mode != "pageable"
    if mode == "pinned_dma":
        monkeypatch.setenv("XRS_HOST_ZC", "0")
    allocs = []

    def hbuf(nbytes):
        if pin:
            p_, a = pinned(nbytes)
            allocs.append(p_)
            return p_, a
        a = np.empty(nbytes, np.uint8)
        return a.ctypes.data, a

    o, x = OracleXRS(D, P), xrs_amd.XRS(D, P)
    stripe = 16 * size
    sp, sbuf = hbuf(n * stripe)  # full stripes: data rows + parity rows
    sbuf[:] = rng.integers(0, 256, size=n * stripe, dtype=np.uint8)
    v = sbuf.reshape(n, 16, size)
    o.encode_batch(v, size, n)
    np_, nbuf = hbuf(n * size)  # new data of the updated row
    nbuf[:] = rng.integers(0, 256, size=n * size, dtype=np.uint8)
    row = 7
    exp = v.copy()
    for s in range(n):
        par = [exp[s, D + r] for r in range(P)]
        o.update(exp[s, row].copy(), nbuf[s * size:(s + 1) * size], row, par)
    x.update_host(sp + row * size, stripe, np_, size, size, row, sp + D * size, size, stripe, n)
    assert np.array_equal(v, exp)
    # Replace rows [3, 9, 0] with data from a separate buffer of 3 rows per stripe
    rows = [3, 9, 0]
    dp, dbuf = hbuf(n * 3 * size)
    dbuf[:] = rng.integers(0, 256, size=n * 3 * size, dtype=np.uint8)
    dv = dbuf.reshape(n, 3, size)
    for s in range(n):
        o.replace([dv[s, i] for i in range(3)], rows, [exp[s, D + r] for r in range(P)])
    x.replace_host(dp, size, 3 * size, rows, size, sp + D * size, size, stripe, n)
    assert np.array_equal(v, exp)
    with pytest.raises(xrs_amd.XRSError, match="illegal data index: 12"):
        x.update_host(sp, stripe, np_, size, size, 12, sp + D * size, size, stripe, n)
    for p_ in allocs:
        xrs_amd.lib().xrs_host_free(p_)


@pytest.mark.parametrize("mode", ["pinned_zero_copy", "pageable"])
def test_reconst_host_negative_single_need_writes_nothing(rng, mode):
    """need = [-1]: xrs.go:238 takes ReconstOne, which rejects k before any
    write ('illegal data index: -1'); the host batch is left unchanged
    (the general path used to run steps 1-2 in place first)."""
    size, n = 4096, 64
    stripe = 16 * size
    if mode == "pageable":
        buf = np.empty(n * stripe, np.uint8)
        ptr = buf.ctypes.data
    else:
        ptr, buf = pinned(n * stripe)
    buf[:] = rng.integers(0, 256, size=n * stripe, dtype=np.uint8)
    v = buf.reshape(n, 16, size)
    OracleXRS(D, P).encode_batch(v, size, n)
    v[:, 3] = 0x5A
    before = buf.copy()
    has = [j for j in range(D + P) if j != 3]
    x = xrs_amd.XRS(D, P)
    with pytest.raises(xrs_amd.XRSError, match="^illegal data index: -1$"):
        x.reconst_host(ptr, size, size, stripe, n, has, [-1])
    assert np.array_equal(buf, before)
    g = xrs_amd.XRSGroup(D, P, [0, 0])
    with pytest.raises(xrs_amd.XRSError, match="^illegal data index: -1$"):
        g.reconst_host(ptr, size, size, stripe, n, has, [-1])
    assert np.array_equal(buf, before)
    if mode != "pageable":
        xrs_amd.lib().xrs_host_free(ptr)
