"""Odd vect sizes (S/2 not a multiple of 16) through the library's OWN staging:
the synchronous per-stripe calls (every staging mode), the batching queue and
the host pipeline all place their staged rows at xrs_batch_layout's base
offset, so the b-halves get the alignment a recommended device batch has.
Every result is compared with the oracle (oracle/xrs_oracle.c).  Reference
semantics: xrs.go:103-128 (Encode), :175-221 (ReconstOne), :236-320
(Reconst), :324-346 (Update), :363-387 (Replace); the size rule is
xrs.go:130-136 (any even size)."""
import ctypes
import threading

import numpy as np
import pytest

import xrs_amd
from oracle.oracle_c import OracleXRS

pytestmark = pytest.mark.gpu
D, P = 12, 4
SIZES = [4100, 4098, (1 << 20) + 2]


def _vects(rng, size):
    return [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(D + P)]


def _check_all_ops(x, o, rng, size):
    """Encode, ReconstOne, 2-lost Reconst, Update, Replace on one stripe."""
    v = _vects(rng, size)
    ref = [a.copy() for a in v]
    o.encode(ref)
    x.encode(v)
    assert all(np.array_equal(a, b) for a, b in zip(v, ref)), "encode"
    k = int(rng.integers(0, D))
    a_need, _ = x.get_need_vects(k)
    w = [a.copy() for a in ref]
    w[k][:] = 0
    for j in range(D + P):  # garbage outside the need set
        if j not in a_need and j != k:
            w[j][: size // 2] = 0xC3
    x.reconst_one(w, k)
    assert np.array_equal(w[k], ref[k]), ("reconst_one", k)
    lost = [k, D + 1 + int(rng.integers(0, P - 1))]
    has = [j for j in range(D + P) if j not in lost]
    g1 = [a.copy() for a in ref]
    for j in lost:
        g1[j][:] = 0x5A
    g2 = [a.copy() for a in g1]
    x.reconst(g1, has, lost)
    o.reconst(g2, has, lost)
    assert all(np.array_equal(a, b) for a, b in zip(g1, g2)), ("reconst", lost)
    row = int(rng.integers(0, D))
    nd = rng.integers(0, 256, size=size, dtype=np.uint8)
    p1 = [a.copy() for a in ref[D:]]
    p2 = [a.copy() for a in ref[D:]]
    x.update(ref[row], nd, row, p1)
    o.update(ref[row], nd, row, p2)
    assert all(np.array_equal(a, b) for a, b in zip(p1, p2)), ("update", row)
    rows = [row, (row + 5) % D]
    data = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in rows]
    x.replace(data, rows, p1)
    o.replace(data, rows, p2)
    assert all(np.array_equal(a, b) for a, b in zip(p1, p2)), ("replace", rows)


@pytest.mark.parametrize("mode", ["zero_copy", "pinned", "direct"])
@pytest.mark.parametrize("size", SIZES)
def test_sync_odd_sizes_every_staging_mode(rng, monkeypatch, size, mode):
    """codec.cpp Stage: zero-copy mirror, pinned mirror + DMA, direct copies."""
    big = str(64 << 20)
    monkeypatch.setenv("XRS_SYNC_ZC_MAX", big if mode == "zero_copy" else "0")
    monkeypatch.setenv("XRS_SYNC_PINNED_MAX", big if mode == "pinned" else "0")
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    for _ in range(3 if size < (1 << 20) else 1):
        _check_all_ops(x, o, rng, size)


@pytest.mark.parametrize("size", SIZES)
def test_queue_odd_sizes_concurrent(size):
    """queue.cpp staging (zero-copy batches below 4 MiB, DMA above): every op
    from several threads at once, each checked against the oracle."""
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    q = xrs_amd.XRSQueue(x, size, max_batch_stripes=16, max_wait_us=50)
    olock = threading.Lock()
    n_threads, per = (8, 4) if size < (1 << 20) else (3, 1)
    errors = []

    def worker(t):
        r = np.random.Generator(np.random.PCG64(700 + t))
        try:
            for i in range(per):
                v = _vects(r, size)
                ref = [a.copy() for a in v]
                with olock:
                    o.encode(ref)
                q.encode(v)
                assert all(np.array_equal(a, b) for a, b in zip(v, ref)), ("enc", t, i)
                k = (t + i) % D
                v[k][:] = 0
                q.reconst_one(v, k)
                assert np.array_equal(v[k], ref[k]), ("rec1", t, i)
                lost = [k, D + 1 + (i % (P - 1))]
                has = [j for j in range(D + P) if j not in lost]
                g1 = [a.copy() for a in ref]
                for j in lost:
                    g1[j][:] = 0x5A
                g2 = [a.copy() for a in g1]
                q.reconst(g1, has, lost)
                with olock:
                    o.reconst(g2, has, lost)
                assert all(np.array_equal(a, b) for a, b in zip(g1, g2)), ("rec", t, i)
                nd = r.integers(0, 256, size=size, dtype=np.uint8)
                p1 = [a.copy() for a in ref[D:]]
                p2 = [a.copy() for a in ref[D:]]
                q.update(ref[k], nd, k, p1)
                with olock:
                    o.update(ref[k], nd, k, p2)
                assert all(np.array_equal(a, b) for a, b in zip(p1, p2)), ("upd", t, i)
                rows = [k, (k + 3) % D]
                data = [r.integers(0, 256, size=size, dtype=np.uint8) for _ in rows]
                q.replace(data, rows, p1)
                with olock:
                    o.replace(data, rows, p2)
                assert all(np.array_equal(a, b) for a, b in zip(p1, p2)), ("rep", t, i)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    q.close()
    assert not errors, errors[:3]
    assert not any(t.is_alive() for t in th)


@pytest.mark.parametrize("size,n", [(4100, 700), (4098, 300), ((1 << 20) + 2, 5)])
def test_host_pipeline_odd_sizes(rng, size, n):
    """codec.cpp run_pipeline / run_pipeline_rows (pageable host batches go
    through the device slots): Encode, ReconstOne, Reconst, Update, Replace."""
    o, x = OracleXRS(D, P), xrs_amd.XRS(D, P)
    stripe = 16 * size
    buf = rng.integers(0, 256, size=n * stripe, dtype=np.uint8)
    v = buf.reshape(n, 16, size)
    ref = v.copy()
    o.encode_batch(ref, size, n)
    x.encode_host(buf.ctypes.data, size, size, stripe, n)
    assert np.array_equal(v, ref)
    k = 5
    v[:, k] = 0
    x.reconst_one_host(buf.ctypes.data, size, size, stripe, n, k)
    assert np.array_equal(v, ref)
    lost = [2, 13]
    has = [j for j in range(D + P) if j not in lost]
    v[:, lost] = 0x5A
    before = v.copy()
    x.reconst_host(buf.ctypes.data, size, size, stripe, n, has, lost)
    for s in sorted({0, n // 2, n - 1}):
        w = [before[s, i].copy() for i in range(D + P)]
        o.reconst(w, has, lost)
        assert np.array_equal(v[s], np.stack(w)), ("reconst", s)
    v[:] = ref
    nbuf = rng.integers(0, 256, size=n * size, dtype=np.uint8)
    row = 7
    exp = v.copy()
    for s in range(n):
        o.update(exp[s, row].copy(), nbuf[s * size:(s + 1) * size], row,
                 [exp[s, D + r] for r in range(P)])
    x.update_host(buf.ctypes.data + row * size, stripe, nbuf.ctypes.data, size, size, row,
                  buf.ctypes.data + D * size, size, stripe, n)
    assert np.array_equal(v, exp)
    rows = [3, 9, 0]
    dbuf = rng.integers(0, 256, size=n * 3 * size, dtype=np.uint8)
    dv = dbuf.reshape(n, 3, size)
    for s in range(n):
        o.replace([dv[s, i] for i in range(3)], rows, [exp[s, D + r] for r in range(P)])
    x.replace_host(dbuf.ctypes.data, size, 3 * size, rows, size, buf.ctypes.data + D * size, size,
                   stripe, n)
    assert np.array_equal(v, exp)


# (vect size, base offset, shard pad, stripe pad): host layouts whose rows sit
# on every address residue mod 4 and whose pitches are not multiples of 4, so
# the pipeline's device image is residue-matched and its copies split into
# pitch groups (codec.cpp copy_rows / plan_image)
ANY_LAYOUTS = [(4098, 0, 0, 0), (4098, 1, 0, 1), (4100, 2, 3, 2), (4100, 3, 5, 3),
               (1026, 1, 1, 0), (1026, 2, 2, 6), (4096, 1, 0, 0), (4096, 0, 2, 2),
               ((1 << 20) + 2, 3, 1, 1), (2, 1, 1, 1)]


@pytest.mark.parametrize("mode", ["pageable", "pinned_dma"])
@pytest.mark.parametrize("size,base_off,shard_pad,stripe_pad", ANY_LAYOUTS)
def test_host_pipeline_any_layout(rng, monkeypatch, size, base_off, shard_pad, stripe_pad, mode):
    """The host copy pipeline on any host layout (xrs_*_host through the
    device slots: pageable memory, or pinned with XRS_HOST_ZC=0): Encode,
    ReconstOne, Reconst (2 lost, retrieveRS side effect), Update from a
    separate odd-strided buffer and Replace(2), every vect vs the oracle and
    every byte outside the vects the call writes unchanged (no widened copy
    writes host memory).  Reference semantics: xrs.go:103-387."""
    if mode == "pinned_dma":
        monkeypatch.setenv("XRS_HOST_ZC", "0")
    o, x, L = OracleXRS(D, P), xrs_amd.XRS(D, P), xrs_amd.lib()
    n = 3 if size > (1 << 16) else 150
    shard, stripe = size + shard_pad, 16 * (size + shard_pad) + stripe_pad
    total = base_off + n * stripe + 64
    pins = []

    def host(nbytes):
        if mode == "pageable":
            a = np.empty(nbytes, np.uint8)
            return a.ctypes.data, a
        p = L.xrs_host_alloc(nbytes)
        assert p
        pins.append(p)
        return p, np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))

    try:
        ptr, buf = host(total)
        buf[:] = rng.integers(0, 256, size=total, dtype=np.uint8)
        base = ptr + base_off

        def at(s, i):
            a = base_off + s * stripe + i * shard
            return slice(a, a + size)

        def vects(b, s):
            return [b[at(s, i)].copy() for i in range(D + P)]

        def check(want, written, what):
            for s in range(n):
                for i in range(D + P):
                    assert np.array_equal(buf[at(s, i)], want[s][i]), (what, s, i)
            mask = np.ones(total, bool)
            for s in range(n):
                for i in written:
                    mask[at(s, i)] = False
            assert np.array_equal(buf[mask], before[mask]), (what, "bytes outside the written vects")

        # Encode
        before = buf.copy()
        want = [vects(buf, s) for s in range(n)]
        for w in want:
            o.encode(w)
        x.encode_host(base, size, shard, stripe, n)
        check(want, range(D, D + P), "encode")
        # ReconstOne(k): vect k zeroed first
        k = 7
        for s in range(n):
            buf[at(s, k)] = 0
        before = buf.copy()
        x.reconst_one_host(base, size, shard, stripe, n, k)
        check(want, [k], "reconst_one")
        # Reconst of data 2 and parity 13, both needed
        lost = [2, 13]
        has = [j for j in range(D + P) if j not in lost]
        for s in range(n):
            for j in lost:
                buf[at(s, j)] = 0x5A
        before = buf.copy()
        want = [vects(buf, s) for s in range(n)]
        for w in want:
            o.reconst(w, has, lost)
        x.reconst_host(base, size, shard, stripe, n, has, lost)
        check(want, range(D + P), "reconst")
        # Update(row) with new data from a separate buffer, odd stride
        row, nstride = 4, size + 3
        nptr, nbuf = host(1 + n * nstride + 8)
        nbuf[:] = rng.integers(0, 256, size=len(nbuf), dtype=np.uint8)
        before = buf.copy()
        want = [vects(buf, s) for s in range(n)]
        for s in range(n):
            new = nbuf[1 + s * nstride:1 + s * nstride + size]
            o.update(want[s][row].copy(), new, row, want[s][D:])
        x.update_host(base + row * shard, stripe, nptr + 1, nstride, size, row,
                      base + D * shard, shard, stripe, n)
        check(want, range(D, D + P), "update")
        # Replace(rows 1, 10) with data from that buffer: 2 vects per stripe
        rows = [1, 10]
        dshard, dstride = size + 1, 2 * (size + 1) + 2
        dptr, dbuf = host(3 + n * dstride + 8)
        dbuf[:] = rng.integers(0, 256, size=len(dbuf), dtype=np.uint8)
        before = buf.copy()
        want = [vects(buf, s) for s in range(n)]
        for s in range(n):
            data = [dbuf[3 + s * dstride + i * dshard:][:size] for i in range(2)]
            o.replace(data, rows, want[s][D:])
        x.replace_host(dptr + 3, dshard, dstride, rows, size, base + D * shard, shard, stripe, n)
        check(want, range(D, D + P), "replace")
    finally:
        for p in pins:
            L.xrs_host_free(p)
