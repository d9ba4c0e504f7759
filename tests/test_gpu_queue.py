"""GPU tests of the batching queue (xrs_queue_*): concurrent per-stripe calls
from many threads, coalesced into device batches, bit-exact to the oracle."""
import ctypes
import threading

import numpy as np
import pytest

import xrs_amd
from oracle.oracle_c import OracleXRS

pytestmark = pytest.mark.gpu
D, P = 12, 4


@pytest.mark.parametrize("size", [4096, 1030, 1 << 20])
def test_queue_concurrent_encode_and_reconst(size):
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    q = xrs_amd.XRSQueue(x, size, max_batch_stripes=64, max_wait_us=100)
    n_threads, per_thread = (16, 24) if size < (1 << 20) else (8, 4)
    errors = []

    def worker(t):
        rng = np.random.Generator(np.random.PCG64(1000 + t))
        try:
            for i in range(per_thread):
                v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(D)]
                v += [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(P)]
                ref = [a.copy() for a in v]
                o.encode(ref)
                q.encode(v)
                assert all(np.array_equal(a, b) for a, b in zip(v, ref)), ("enc", t, i)
                k = int(rng.integers(0, D))
                a_need, b_need = x.get_need_vects(k)
                v[k][:] = 0
                for j in range(D + P):  # garbage outside the need set
                    if j not in a_need and j != k:
                        v[j][: size // 2] = 0xC3
                q.reconst_one(v, k)
                assert np.array_equal(v[k], ref[k]), ("rec", t, i, k)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    q.close()
    assert not errors, errors[:3]


def test_queue_errors():
    x = xrs_amd.XRS(D, P)
    q = xrs_amd.XRSQueue(x, 64)
    with pytest.raises(xrs_amd.XRSError, match="illegal data index: 12"):
        q.reconst_one([np.zeros(64, np.uint8) for _ in range(16)], 12)
    with pytest.raises(xrs_amd.XRSError, match="illegal vects"):
        q.encode([np.zeros(64, np.uint8) for _ in range(15)])
    with pytest.raises(xrs_amd.XRSError):
        xrs_amd.XRSQueue(x, 63)
    q.close()


@pytest.mark.parametrize("size", [4096, 384 << 10, (4 << 20) + 2])
def test_sync_calls_from_many_threads(size):
    """The per-stripe sync API on ONE codec from many threads at once (every
    staging mode: zero-copy, pinned, direct): every call of every kind is
    bit-exact to the oracle (the codec is shared, its staging is not racy)."""
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    n_threads, per_thread = (8, 6) if size <= (1 << 20) else (4, 1)
    errors = []

    def worker(t):
        rng = np.random.Generator(np.random.PCG64(2000 + t))
        try:
            for i in range(per_thread):
                v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(D + P)]
                ref = [a.copy() for a in v]
                o.encode(ref)
                x.encode(v)
                assert all(np.array_equal(a, b) for a, b in zip(v, ref)), ("enc", t, i)
                lost = [int(j) for j in rng.permutation(D + P)[:3]]
                has = [j for j in range(D + P) if j not in lost]
                r1, r2 = [a.copy() for a in v], [a.copy() for a in v]
                for j in lost:
                    r1[j][:] = 0
                    r2[j][:] = 0
                x.reconst(r1, has, lost)
                o.reconst(r2, has, lost)
                assert all(np.array_equal(a, b) for a, b in zip(r1, r2)), ("rec", t, i)
                row = int(rng.integers(0, D))
                new = rng.integers(0, 256, size=size, dtype=np.uint8)
                p1, p2 = [a.copy() for a in v[D:]], [a.copy() for a in v[D:]]
                x.update(v[row], new, row, p1)
                o.update(v[row], new, row, p2)
                assert all(np.array_equal(a, b) for a, b in zip(p1, p2)), ("upd", t, i)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:3]


def test_queue_close_while_callers_in_flight():
    """close() while 16 threads keep submitting: every call either returns a
    bit-exact result or raises (the queue is closed); none hangs, and the
    queue is torn down only after the last call has left."""
    size = 4096
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    q = xrs_amd.XRSQueue(x, size, max_batch_stripes=64, max_wait_us=200)
    ok, closed, bad = [0], [0], []
    lock = threading.Lock()
    go = threading.Event()

    def worker(t):
        rng = np.random.Generator(np.random.PCG64(3000 + t))
        go.wait()
        for i in range(1 << 30):  # until the queue is closed
            v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(D + P)]
            ref = [a.copy() for a in v]
            o.encode(ref)
            try:
                q.encode(v)
            except xrs_amd.XRSError:
                with lock:
                    closed[0] += 1
                return
            if not all(np.array_equal(a, b) for a, b in zip(v, ref)):
                bad.append((t, i))
            with lock:
                ok[0] += 1

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for t in th:
        t.start()
    go.set()
    import time
    time.sleep(0.3)
    q.close()
    for t in th:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in th), "a caller hung after close()"
    assert not bad, bad[:3]
    assert ok[0] > 0 and closed[0] > 0, (ok[0], closed[0])


@pytest.mark.parametrize("size,d,p", [(4096, 12, 4), (1030, 12, 4), (4096, 1, 2), (65536, 6, 3)])
def test_queue_concurrent_update(size, d, p):
    """xrs_queue_update from many threads (rows differ: one batch carries
    every row, update_rows kernel) interleaved with Encode and ReconstOne on
    the same queue: parity bit-exact to the oracle after every call."""
    x, o = xrs_amd.XRS(d, p), OracleXRS(d, p)
    q = xrs_amd.XRSQueue(x, size, max_batch_stripes=32, max_wait_us=100)
    errors = []

    def worker(t):
        rng = np.random.Generator(np.random.PCG64(4000 + t))
        try:
            v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(d + p)]
            q.encode(v)
            ref = [a.copy() for a in v]
            o.encode(ref)
            assert all(np.array_equal(a, b) for a, b in zip(v, ref)), ("enc", t)
            for i in range(12):
                row = int(rng.integers(0, d))
                new = rng.integers(0, 256, size=size, dtype=np.uint8)
                q.update(v[row], new, row, v[d:])
                o.update(ref[row], new, row, ref[d:])
                v[row][:] = new
                ref[row][:] = new
                assert all(np.array_equal(a, b) for a, b in zip(v[d:], ref[d:])), ("upd", t, i)
                if i % 4 == 3:
                    k = int(rng.integers(0, d))
                    w = [a.copy() for a in v]
                    w[k][:] = 0
                    q.reconst_one(w, k)
                    assert np.array_equal(w[k], v[k]), ("rec", t, i)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(12)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    q.close()
    assert not errors, errors[:3]
    with pytest.raises(xrs_amd.XRSError, match="illegal data index"):
        xrs_amd.XRSQueue(x, size).update(np.zeros(size, np.uint8), np.zeros(size, np.uint8), d,
                                         [np.zeros(size, np.uint8) for _ in range(p)])


def test_batched_calls_from_threads_on_own_streams():
    """One codec, 6 host threads, each launching batched Encode / ReconstOne /
    Update on its own HIP stream and buffer at once (the codec is immutable
    after xrs_new; batched calls share no staging): every result bit-exact."""
    torch = pytest.importorskip("torch")
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    size, n = 4096, 300
    errors = []

    def worker(t):
        try:
            rng = np.random.Generator(np.random.PCG64(5000 + t))
            host = rng.integers(0, 256, size=(n, D + P, size), dtype=np.uint8)
            ref = host.copy()
            o.encode_batch(ref, size, n)
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                dt = torch.from_numpy(host).cuda()
                s = st.cuda_stream
                for it in range(5):
                    x.encode_batched(dt.data_ptr(), size, size, (D + P) * size, n, s)
                    k = (t + it) % D
                    dt[:, k].zero_()
                    x.reconst_one_batched(dt.data_ptr(), size, size, (D + P) * size, n, k, s)
                st.synchronize()
                assert np.array_equal(dt.cpu().numpy(), ref), t
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:3]


@pytest.mark.parametrize("size", [4096, 1030])
def test_queue_reconst_patterns(size):
    """xrs_queue_reconst from 12 threads over 3 loss patterns (batches keyed by
    pattern), plus unclean calls (repeated index, need inside dpHas) that run
    as plain xrs_reconst: every buffer, side effects included, equals the
    oracle's."""
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    q = xrs_amd.XRSQueue(x, size, max_batch_stripes=32, max_wait_us=200)
    patterns = [([0, 1], [0, 1]), ([3, 13, 15], [3, 13]), ([2, 5, 9, 14], [2, 5, 9, 14]),
                ([7], [7, 7]), ([1, 4], [1, 2])]
    errors = []

    def worker(t):
        rng = np.random.Generator(np.random.PCG64(6000 + t))
        try:
            for i in range(10):
                lost, need = patterns[(t + i) % len(patterns)]
                v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(D + P)]
                o.encode(v)
                has = [j for j in range(D + P) if j not in lost]
                for j in lost:
                    v[j][:] = 0x5A
                a, b = [r.copy() for r in v], [r.copy() for r in v]
                q.reconst(a, has, need)
                o.reconst(b, has, need)
                assert all(np.array_equal(s, u) for s, u in zip(a, b)), (t, i, lost, need)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(12)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    st = q.stats()
    q.close()
    assert not errors, errors[:3]
    assert st["stripes"] > 0


def test_queue_replace_rows_sets():
    """xrs_queue_replace from 10 threads over 3 rows sets (one batch per set):
    parity bit-exact to the oracle; bad rows rejected before any write."""
    size = 4096
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    q = xrs_amd.XRSQueue(x, size, max_batch_stripes=32, max_wait_us=200)
    sets = [[0], [1, 4, 7, 10], [11, 2, 5, 8, 3, 6, 9, 0]]
    errors = []

    def worker(t):
        rng = np.random.Generator(np.random.PCG64(6500 + t))
        try:
            for i in range(8):
                rows = sets[(t + i) % len(sets)]
                v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(D + P)]
                o.encode(v)
                data = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in rows]
                p1, p2 = [a.copy() for a in v[D:]], [a.copy() for a in v[D:]]
                q.replace(data, rows, p1)
                o.replace(data, rows, p2)
                assert all(np.array_equal(a, b) for a, b in zip(p1, p2)), (t, i, rows)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(10)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    par = [np.zeros(size, np.uint8) for _ in range(P)]
    with pytest.raises(xrs_amd.XRSError, match="illegal data index: 12"):
        q.replace([np.zeros(size, np.uint8)], [12], par)
    assert not any(a.any() for a in par)
    q.close()
    assert not errors, errors[:3]


@pytest.mark.parametrize("d,p,size", [(12, 4, 4096), (6, 3, 1030), (10, 4, 65536)])
def test_queue_mixed_ops_fuzz(d, p, size):
    """16 threads issue random operations of every kind (Encode, ReconstOne,
    Reconst over a few loss patterns, Update of any row, Replace over a few
    rows sets) on one queue, so batches of different kinds and patterns
    open and close under contention; every result equals the oracle's."""
    x, o = xrs_amd.XRS(d, p), OracleXRS(d, p)
    q = xrs_amd.XRSQueue(x, size, max_batch_stripes=16, max_wait_us=80)
    rng0 = np.random.Generator(np.random.PCG64(77 + d))
    patterns = []
    for _ in range(3):
        lost = [int(v) for v in rng0.permutation(d + p)[: int(rng0.integers(2, p + 1))]]
        patterns.append((lost, lost[: max(2, len(lost) - 1)]))
    row_sets = [[int(v) for v in rng0.permutation(d)[: int(rng0.integers(1, d + 1))]]
                for _ in range(3)]
    errors = []

    def worker(t):
        rng = np.random.Generator(np.random.PCG64(8000 + t))
        try:
            for i in range(10):
                v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(d + p)]
                o.encode(v)
                a, b = [r.copy() for r in v], [r.copy() for r in v]
                op = int(rng.integers(0, 5))
                if op == 0:
                    for r in a[d:]:
                        r[:] = 0
                    q.encode(a)
                elif op == 1:
                    k = int(rng.integers(0, d))
                    a[k][:] = 0
                    q.reconst_one(a, k)
                elif op == 2:
                    lost, need = patterns[int(rng.integers(0, len(patterns)))]
                    has = [j for j in range(d + p) if j not in lost]
                    for j in lost:
                        a[j][:] = 0x11
                        b[j][:] = 0x11
                    q.reconst(a, has, need)
                    o.reconst(b, has, need)
                elif op == 3:
                    row = int(rng.integers(0, d))
                    new = rng.integers(0, 256, size=size, dtype=np.uint8)
                    q.update(a[row], new, row, a[d:])
                    o.update(b[row], new, row, b[d:])
                else:
                    rows = row_sets[int(rng.integers(0, len(row_sets)))]
                    data = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in rows]
                    q.replace(data, rows, a[d:])
                    o.replace(data, rows, b[d:])
                assert all(np.array_equal(s, u) for s, u in zip(a, b)), (t, i, op)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    q.close()
    assert not errors, errors[:3]


@pytest.mark.parametrize("env", [
    {"XRS_QUEUE_INFLIGHT": "1"},
    {"XRS_QUEUE_INFLIGHT": "8", "XRS_QUEUE_BATCHES": "10"},
    {"XRS_QUEUE_WORKERS": "3"},
    {"XRS_QUEUE_POLICY": "timer"},
    {"XRS_QUEUE_ZC_MAX": "0"},  # every batch through H2D / kernel / D2H
])
def test_queue_policies_bit_exact(env, monkeypatch):
    """The queue's knobs (read at xrs_queue_new) change batching, never
    results: Encode + ReconstOne from 24 threads, bit-exact to the oracle,
    and every staging batch FREE again afterwards (xrs_queue_dump)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    size = 4096
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    q = xrs_amd.XRSQueue(x, size, max_batch_stripes=16, max_wait_us=50)
    errors = []

    def worker(t):
        rng = np.random.Generator(np.random.PCG64(5000 + t))
        try:
            for i in range(12):
                v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(D + P)]
                ref = [a.copy() for a in v]
                o.encode(ref)
                q.encode(v)
                assert all(np.array_equal(a, b) for a, b in zip(v, ref)), ("enc", t, i)
                k = int(rng.integers(0, D))
                v[k][:] = 0x77
                q.reconst_one(v, k)
                assert np.array_equal(v[k], ref[k]), ("rec", t, i, k)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(24)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "a caller hung:\n" + q.dump()
    assert not errors, errors[:3]
    st = q.stats()
    assert st["stripes"] == 24 * 12 * 2, st
    dump = q.dump()
    batches = [ln for ln in dump.splitlines() if ln.startswith("batch ")]
    assert batches and all(" FREE " in ln for ln in batches), dump
    assert "in_flight 0" in dump and "active 0" in dump, dump
    q.close()


@pytest.mark.parametrize("size", [4096, 1030, 65536, 1 << 20])
def test_shared_codec_concurrent_sync_calls(size):
    """The plain per-stripe calls (x.encode / update / reconst_one /
    reconst / replace, the cgo shim's path) from 16 threads on ONE codec: contended calls go through
    the codec's automatic queue (codec.cpp auto_queue), the rest run
    directly; every result is bit-exact to the oracle."""
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    errors = []
    olock = threading.Lock()

    def worker(t):
        rng = np.random.Generator(np.random.PCG64(7000 + t))
        try:
            for i in range(10 if size < (1 << 20) else 3):
                v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(D + P)]
                ref = [a.copy() for a in v]
                with olock:
                    o.encode(ref)
                x.encode(v)
                assert all(np.array_equal(a, b) for a, b in zip(v, ref)), ("enc", t, i)
                row = int(rng.integers(0, D))
                new = rng.integers(0, 256, size=size, dtype=np.uint8)
                ref2 = [a.copy() for a in ref]
                ref2[row] = new.copy()
                with olock:
                    o.encode(ref2)
                par = v[D:]
                x.update(v[row], new, row, par)
                assert all(np.array_equal(a, b) for a, b in zip(par, ref2[D:])), ("upd", t, i)
                v[row] = new
                k = int(rng.integers(0, D))
                v[k][:] = 0
                x.reconst_one(v, k)
                assert np.array_equal(v[k], ref2[k]), ("rec", t, i, k)
                # Reconst of one data and one parity vect (both needed): the
                # reference's side effects on surviving parity included
                lost = [k, D + 1 + i % (P - 1)]
                has = [j for j in range(D + P) if j not in lost]
                g1 = [a.copy() for a in v]
                g2 = [a.copy() for a in v]
                for j in lost:
                    g1[j][:] = 0x5A
                    g2[j][:] = 0x5A
                with olock:
                    o.reconst(g2, has, lost)
                x.reconst(g1, has, lost)
                assert all(np.array_equal(a, b) for a, b in zip(g1, g2)), ("reconst", t, i)
                # Replace of two rows with fresh data
                rows = [row, (row + 5) % D]
                nd = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in rows]
                pq = [a.copy() for a in v[D:]]
                ps = [a.copy() for a in v[D:]]
                with olock:
                    o.replace(nd, rows, ps)
                x.replace(nd, rows, pq)
                assert all(np.array_equal(a, b) for a, b in zip(pq, ps)), ("replace", t, i)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "a caller hung"
    assert not errors, errors[:3]


def test_queue_coalesces_barrier_released_callers():
    """32 threads released together by a barrier, each making one 4 KiB
    Encode and then one ReconstOne call per round on ONE queue (the
    reference's per-stripe call pattern, xrs_test.go:498-521): the queue runs
    them in fewer batches than calls (xrs_queue_batch_sizes), and every call
    is bit-exact to the oracle.  The calls go straight to the C ABI with
    their pointer arrays made beforehand, but Python threads still reach it
    one GIL hand-off apart, about as far apart as a one-stripe batch takes to
    run, so most batches stay small here (measured: 384 calls in 297-343
    batches of up to 4-5 stripes).  The C++ port's TestQueue_Coalesces
    (tests/cpp/xrs_test.cpp, native threads) asserts fewer than half as many
    batches as calls and several of 4 stripes or more."""
    size, n_threads, rounds = 4096, 32, 6
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    q = xrs_amd.XRSQueue(x, size)
    L, h = xrs_amd.lib(), q.handle
    rng = np.random.Generator(np.random.PCG64(9100))
    work = []
    for t in range(n_threads):
        per = []
        for r in range(rounds):
            v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(D + P)]
            ref = [a.copy() for a in v]
            o.encode(ref)
            arr = (ctypes.c_void_p * (D + P))(*[a.ctypes.data for a in v])
            per.append((v, ref, int(rng.integers(0, D)), arr))
        work.append(per)
    bar = threading.Barrier(n_threads)
    errors = []

    def worker(t):
        try:
            for r, (v, ref, k, arr) in enumerate(work[t]):
                bar.wait(timeout=60)
                assert L.xrs_queue_encode(h, arr, D + P) == 0, ("enc rc", t, r)
                assert all(np.array_equal(a, b) for a, b in zip(v, ref)), ("enc", t, r)
                v[k][:] = 0x3C
                bar.wait(timeout=60)
                assert L.xrs_queue_reconst_one(h, arr, D + P, k) == 0, ("rec rc", t, r)
                assert np.array_equal(v[k], ref[k]), ("rec", t, r, k)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))
            bar.abort()

    th = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "a caller hung:\n" + q.dump()
    st, sizes = q.stats(), q.batch_sizes()
    q.close()
    assert not errors, errors[:3]
    calls = n_threads * rounds * 2
    print(f"queue: {calls} calls in {st['batches']} batches, stripes per batch {sizes}")
    assert st["stripes"] == calls, st
    assert sum(n * c for n, c in sizes.items()) == calls, sizes
    assert st["batches"] < calls and max(sizes) >= 2, (st, sizes)
