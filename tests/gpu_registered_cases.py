"""Cases of tests/test_gpu_registered.py (each function runs in a child
pytest process; see there why).  GPU tests of the per-stripe calls on
caller-registered host memory: vects
inside ranges pinned and mapped by xrs_host_alloc / xrs_host_register run
without the CPU gather / scatter through pinned staging -- in place over PCIe
for a lone sync call (codec.cpp reg_vects), and for coalesced calls through
one launch of the indirect-row kernels (pair_ind_kernel, rows_ind_kernel,
update_rows_ind_kernel) over the queue's per-batch row address table
(queue.cpp table mode).
Every result, side effects included, is compared with the oracle
(oracle/xrs_oracle.c, following xrs.go:103-387)."""
import ctypes
import os
import threading

import numpy as np
import pytest

import xrs_amd
from oracle.oracle_c import OracleXRS

pytestmark = pytest.mark.gpu


D, P = 12, 4
PAGE = 4096


class Arena:
    """Host memory the library knows as pinned and mapped: `alloc` from
    xrs_host_alloc, `register` a numpy buffer passed to xrs_host_register.
    take(n, skew) hands out n-byte vects, each starting `skew` bytes past a
    16-byte boundary (Go slices and numpy views need not be aligned)."""

    def __init__(self, nbytes, kind):
        self.kind = kind
        L = xrs_amd.lib()
        if kind == "alloc":
            self.ptr = L.xrs_host_alloc(nbytes)
            assert self.ptr
            self.buf = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(self.ptr))
        else:
            # whole pages (HIP pins pages), all inside this buffer, so no page
            # another object shares is pinned with it
            nbytes = (nbytes + PAGE - 1) // PAGE * PAGE
            raw = np.empty(nbytes + PAGE, np.uint8)
            off = (-raw.ctypes.data) % PAGE
            self.raw = raw
            self.buf = raw[off:off + nbytes]
            self.ptr = self.buf.ctypes.data
            assert L.xrs_host_register(self.ptr, nbytes) == 0
        self.pos = 0
        self.taken = []

    def take(self, n, skew=0):
        start = (self.pos + 15) // 16 * 16 + skew
        assert start + n <= len(self.buf), "arena too small"
        self.pos = start + n
        self.taken.append((start, start + n))
        return self.buf[start:start + n]

    def canary(self, byte=0xC5):
        """Fill the whole arena (before any take) with `byte`."""
        self.buf[:] = byte
        self.canary_byte = byte

    def untouched(self):
        """Offsets outside every taken vect whose canary byte changed."""
        mask = np.ones(len(self.buf), bool)
        for a, b in self.taken:
            mask[a:b] = False
        return np.nonzero(mask & (self.buf != self.canary_byte))[0]

    def close(self):
        L = xrs_amd.lib()
        if self.kind == "alloc":
            L.xrs_host_free(self.ptr)
        else:
            assert L.xrs_host_unregister(self.ptr) == 0
            # the pages go back to numpy's allocator (a Go BufPool.Close()
            # followed by GC); later buffers and the runtime's
            # pageable copies may land on them
        self.raw = self.buf = None


def _ind_launches(tr):
    """Launches of the indirect-row kernels in a traced_kernels() dict."""
    return sum(n for k, n in tr.items() if "_ind_kernel" in k)


def _fill(rng, arrs):
    for a in arrs:
        a[:] = rng.integers(0, 256, size=len(a), dtype=np.uint8)


def _same(a, b):
    return all(np.array_equal(x, y) for x, y in zip(a, b))


@pytest.mark.parametrize("size", [4096, 4098, 1 << 20])
@pytest.mark.parametrize("kind,skew", [("alloc", 0), ("register", 3)])
def test_sync_calls_in_place(size, kind, skew):
    """All five per-stripe calls on registered vects run in place (the trace
    records host:sync_in_place once per call) and equal the oracle, the
    reference's Reconst side effects on surviving parity included."""
    rng = np.random.Generator(np.random.PCG64(size + skew))
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    ar = Arena(24 * (size + 32), kind)
    try:
        v = [ar.take(size, skew) for _ in range(D + P)]
        extra = [ar.take(size, skew) for _ in range(3)]
        _fill(rng, v + extra)
        xrs_amd.trace_kernels(True)
        # Encode (xrs.go:103)
        ref = [a.copy() for a in v]
        o.encode(ref)
        x.encode(v)
        assert _same(v, ref), "encode"
        # ReconstOne (xrs.go:175): vects outside the need set hold garbage
        k = 7
        a_need, b_need = x.get_need_vects(k)
        for j in range(D + P):
            if j != k and j not in a_need:
                v[j][: size // 2] = 0xC3
        v[k][:] = 0
        x.reconst_one(v, k)
        assert np.array_equal(v[k], ref[k]), "reconst_one"
        for j in range(D + P):
            v[j][:] = ref[j]
        # Reconst (xrs.go:236) of two data vects and one piggybacked parity
        lost = [1, 10, D + 2]
        has = [j for j in range(D + P) if j not in lost]
        for j in lost:
            v[j][:] = 0x5A
        want = [a.copy() for a in v]
        o.reconst(want, has, lost)
        x.reconst(v, has, lost)
        assert _same(v, want), "reconst"
        for j in range(D + P):
            v[j][:] = ref[j]
        # Update (xrs.go:324) of row 4 with new bytes
        new = extra[0]
        par = [a.copy() for a in ref[D:]]
        o.update(ref[4], new, 4, par)
        x.update(v[4], new, 4, v[D:])
        assert _same(v[D:], par), "update"
        # Replace (xrs.go:363) of rows 2 and 9 (zero -> data direction)
        rows = [2, 9]
        par2 = [a.copy() for a in v[D:]]
        o.replace([extra[1], extra[2]], rows, par2)
        x.replace([extra[1], extra[2]], rows, v[D:])
        assert _same(v[D:], par2), "replace"
        xrs_amd.trace_kernels(False)
        tr = xrs_amd.traced_kernels()
        assert tr.get("host:sync_in_place") == 5, tr
    finally:
        xrs_amd.trace_kernels(False)
        ar.close()


def test_sync_partly_registered_falls_back():
    """A call with one vect outside registered memory copies as before (same
    result, no in-place trace event); ReconstOne needs only its need set and
    vect k registered."""
    size = 4096
    rng = np.random.Generator(np.random.PCG64(11))
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    ar = Arena(20 * (size + 32), "alloc")
    try:
        v = [ar.take(size) for _ in range(D + P)]
        _fill(rng, v)
        plain = np.array(v[3])  # ordinary pageable memory
        mixed = v[:3] + [plain] + v[4:]
        ref = [a.copy() for a in mixed]
        o.encode(ref)
        xrs_amd.trace_kernels(True)
        x.encode(mixed)
        assert _same(mixed, ref)
        assert "host:sync_in_place" not in xrs_amd.traced_kernels()
        # ReconstOne(8) reads only its need set (xrs.go:146-171): b-halves of
        # 0..11 but 8 and of 12 and 15 (bi), a-halves of 2, 5 and 11; vects 13
        # and 14 are never read, so they may live anywhere
        a_need, b_need = x.get_need_vects(8)
        assert a_need == [2, 5, 11] and b_need == [12, 15], (a_need, b_need)
        w = list(v)
        for j in range(D + P):
            w[j][:] = ref[j]
        w[13] = np.array(ref[13])
        w[14] = None
        w[8][:] = 0
        xrs_amd.trace_kernels(True)
        x.reconst_one([a if a is not None else np.zeros(size, np.uint8) for a in w], 8)
        assert np.array_equal(w[8], ref[8])
        assert xrs_amd.traced_kernels().get("host:sync_in_place") == 1
        # a pageable vect inside the need set: the call copies
        w[0] = np.array(ref[0])
        w[8][:] = 0
        xrs_amd.trace_kernels(True)
        x.reconst_one([a if a is not None else np.zeros(size, np.uint8) for a in w], 8)
        assert np.array_equal(w[8], ref[8])
        assert "host:sync_in_place" not in xrs_amd.traced_kernels()
    finally:
        xrs_amd.trace_kernels(False)
        ar.close()


@pytest.mark.parametrize("size", [4096, 4098, 65536])
def test_queue_registered_and_plain_callers(size):
    """24 threads on one queue, barrier-released per round, every op kind
    (Encode, ReconstOne, Reconst of one pattern, Update, Replace of one rows
    set); even threads use registered vects, odd ones plain numpy, so batches
    mix both (the table points the plain slots at their pinned staging rows).
    Every call equals the oracle; the indirect-row kernels ran."""
    n_th, rounds = 24, 3
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    q = xrs_amd.XRSQueue(x, size, max_batch_stripes=64)
    ar = Arena(n_th * 20 * (size + 32), "alloc")
    lost, need = [0, 5, D + 1], [0, 5, D + 1]
    has = [j for j in range(D + P) if j not in lost]
    rows = [3, 8]
    work = []
    for t in range(n_th):
        rng = np.random.Generator(np.random.PCG64(500 + t))
        if t % 2 == 0:
            v = [ar.take(size, t % 5) for _ in range(D + P)]
            ex = [ar.take(size, t % 5) for _ in range(3)]
        else:
            v = [np.empty(size, np.uint8) for _ in range(D + P)]
            ex = [np.empty(size, np.uint8) for _ in range(3)]
        work.append((rng, v, ex))
    bar = threading.Barrier(n_th)
    olock = threading.Lock()
    errors = []

    def worker(t):
        rng, v, ex = work[t]
        try:
            for r in range(rounds):
                _fill(rng, v + ex)
                ref = [a.copy() for a in v]
                with olock:
                    o.encode(ref)
                bar.wait(timeout=60)
                q.encode(v)
                assert _same(v, ref), ("enc", t, r)
                k = (t + r) % D
                v[k][:] = 0
                bar.wait(timeout=60)
                q.reconst_one(v, k)
                assert np.array_equal(v[k], ref[k]), ("rec1", t, r)
                for j in lost:
                    v[j][:] = 0x11
                want = [a.copy() for a in v]
                with olock:
                    o.reconst(want, has, need)
                bar.wait(timeout=60)
                q.reconst(v, has, need)
                assert _same(v, want), ("rec", t, r)
                for j in range(D + P):
                    v[j][:] = ref[j]
                par = [a.copy() for a in ref[D:]]
                with olock:
                    o.update(ref[t % D], ex[0], t % D, par)
                bar.wait(timeout=60)
                q.update(v[t % D], ex[0], t % D, v[D:])
                assert _same(v[D:], par), ("upd", t, r)
                par2 = [a.copy() for a in v[D:]]
                with olock:
                    o.replace([ex[1], ex[2]], rows, par2)
                bar.wait(timeout=60)
                q.replace([ex[1], ex[2]], rows, v[D:])
                assert _same(v[D:], par2), ("rep", t, r)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))
            bar.abort()

    xrs_amd.trace_kernels(True)
    th = [threading.Thread(target=worker, args=(t,)) for t in range(n_th)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=180)
    xrs_amd.trace_kernels(False)
    alive = any(t.is_alive() for t in th)
    st = q.stats()
    dump = q.dump() if alive else ""
    q.close()
    ar.close()
    assert not alive, "a caller hung:\n" + dump
    assert not errors, errors[:3]
    assert st["stripes"] == n_th * rounds * 5, st
    tr = xrs_amd.traced_kernels()
    assert _ind_launches(tr) > 0, tr


def test_shared_codec_registered_concurrent():
    """The plain per-stripe calls from 16 threads on ONE codec with
    registered vects: the lone caller runs in place, contended calls go
    through the codec's automatic queue in table mode; bit-exact."""
    size = 4096
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    ar = Arena(16 * 18 * (size + 32), "register")
    errors = []
    olock = threading.Lock()
    vs = [([ar.take(size, 8) for _ in range(D + P)], ar.take(size, 8)) for _ in range(16)]

    def worker(t):
        rng = np.random.Generator(np.random.PCG64(900 + t))
        v, new = vs[t]
        try:
            for i in range(12):
                _fill(rng, v + [new])
                ref = [a.copy() for a in v]
                with olock:
                    o.encode(ref)
                x.encode(v)
                assert _same(v, ref), ("enc", t, i)
                k = (t + i) % D
                v[k][:] = 0
                x.reconst_one(v, k)
                assert np.array_equal(v[k], ref[k]), ("rec", t, i)
                par = [a.copy() for a in ref[D:]]
                with olock:
                    o.update(ref[k], new, k, par)
                x.update(v[k], new, k, v[D:])
                assert _same(v[D:], par), ("upd", t, i)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    xrs_amd.trace_kernels(True)
    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    xrs_amd.trace_kernels(False)
    alive = any(t.is_alive() for t in th)
    ar.close()
    assert not alive, "a caller hung"
    assert not errors, errors[:3]
    tr = xrs_amd.traced_kernels()
    assert tr.get("host:sync_in_place", 0) + _ind_launches(tr) > 0, tr


FUZZ_CODECS = [(12, 4), (10, 4), (6, 3), (4, 2), (5, 5), (20, 4), (1, 2), (30, 6), (3, 9), (16, 8)]
FUZZ_OPS = ["encode", "reconst_one", "reconst", "update", "replace"]


@pytest.mark.parametrize("seed", range(int(os.environ.get("XRS_FUZZ_SEEDS", "4"))))
@pytest.mark.parametrize("via", ["sync", "queue"])
def test_registered_fuzz_vs_oracle(seed, via):
    """Random codecs, sizes, per-vect skews and operations on registered
    vects, through the in-place sync calls or a queue (table mode: the
    indirect-row kernels, chained launches past 24 sources included), against
    the oracle applied to copies; every vect is compared, side effects
    included."""
    rng = np.random.Generator(np.random.PCG64(7700 + seed + (0 if via == "sync" else 50000)))
    xrs_amd.trace_kernels(True)
    try:
        for case in range(12):
            d, p = FUZZ_CODECS[int(rng.integers(0, len(FUZZ_CODECS)))]
            size = int(rng.choice([2, 34, 4096, 4112, 65538]))
            x, o = xrs_amd.XRS(d, p), OracleXRS(d, p)
            ar = Arena((2 * d + p + 2) * (size + 32), "alloc")
            ar.canary()  # nothing outside the vects may be written
            q = xrs_amd.XRSQueue(x, size) if via == "queue" else None
            api = q if q is not None else x
            try:
                def take(count):
                    out = [ar.take(size, int(rng.integers(0, 16))) for _ in range(count)]
                    _fill(rng, out)
                    return out

                a = take(d + p)
                o.encode(a)
                b = [t.copy() for t in a]
                op = FUZZ_OPS[int(rng.integers(0, len(FUZZ_OPS)))]
                tag = (seed, case, d, p, size, op, via)
                if op == "encode":
                    for t in a[d:]:
                        t[:] = 0x33
                    api.encode(a)
                elif op == "reconst_one":
                    k = int(rng.integers(0, d))
                    a[k][:] = 0
                    api.reconst_one(a, k)
                elif op == "reconst":
                    lost = [int(t) for t in rng.permutation(d + p)[: int(rng.integers(1, p + 1))]]
                    need = lost[: int(rng.integers(1, len(lost) + 1))]
                    has = [i for i in range(d + p) if i not in lost]
                    for i in lost:
                        a[i][:] = 0xA5
                        b[i][:] = 0xA5
                    api.reconst(a, has, need)
                    o.reconst(b, has, need)
                elif op == "update":
                    row = int(rng.integers(0, d))
                    new = take(1)[0]
                    api.update(a[row], new, row, a[d:])
                    o.update(b[row], new, row, b[d:])
                else:
                    k = int(rng.integers(1, d + 1))
                    rows = [int(t) for t in rng.permutation(d)[:k]]
                    data = take(k)
                    api.replace(data, rows, a[d:])
                    o.replace(data, rows, b[d:])
                for j, (s_, t_) in enumerate(zip(a, b)):
                    if not np.array_equal(s_, t_):
                        bad = np.nonzero(s_ != t_)[0]
                        raise AssertionError(f"{tag}: vect {j}: {len(bad)} bytes differ, first at {bad[0]}")
                stray = ar.untouched()
                assert len(stray) == 0, f"{tag}: {len(stray)} bytes outside the vects written, first at {stray[0]} " \
                    f"(vects at {ar.taken})"
            finally:
                if q is not None:
                    q.close()
                ar.close()
    finally:
        xrs_amd.trace_kernels(False)
    tr = xrs_amd.traced_kernels()
    if via == "queue":
        assert _ind_launches(tr) > 0, tr
    else:
        assert tr.get("host:sync_in_place", 0) > 0, tr


@pytest.mark.parametrize("nbytes", [64 << 10, 2 << 20])
def test_unregister_free_reuse_then_pageable_copy(nbytes):
    """register -> in-place Encode -> unregister -> free -> the allocator hands
    the pages out again -> PyTorch's pageable copies from and into them.
    Bytes exact, no HIP error; the C++ twin is tests/cpp/xrs_test.cpp
    TestRegistered_UnregisterFreeReuse.  Reference call on the pooled
    buffers: xrs.go:103-128."""
    import gc

    import torch

    L = xrs_amd.lib()
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    rng = np.random.Generator(np.random.PCG64(nbytes))
    size = 4096
    reused = 0
    for rnd in range(6):
        raw = np.empty(nbytes + PAGE, np.uint8)
        buf = raw[(-raw.ctypes.data) % PAGE:][:nbytes]
        lo, hi = buf.ctypes.data, buf.ctypes.data + nbytes
        assert L.xrs_host_register(lo, nbytes) == 0
        v = [buf[i * size:(i + 1) * size] for i in range(D + P)]
        buf[:D * size] = rng.integers(0, 256, size=D * size, dtype=np.uint8)
        want = [np.array(w) for w in v]
        o.encode(want)
        x.encode(v)  # in place over PCIe (registered)
        assert all(np.array_equal(w, c) for w, c in zip(v, want))
        assert L.xrs_host_unregister(lo) == 0
        del v, buf, raw
        gc.collect()
        held, hit = [], None
        for _ in range(16):
            b = np.empty(nbytes + PAGE, np.uint8)
            if b.ctypes.data < hi and lo < b.ctypes.data + b.nbytes:
                hit = b
                break
            held.append(b)
        reused += hit is not None
        b = hit if hit is not None else np.empty(nbytes + PAGE, np.uint8)
        del held, hit
        b[:] = rng.integers(0, 256, size=b.nbytes, dtype=np.uint8)
        t = torch.from_numpy(b).to("cuda:0")  # pageable H2D from the reused pages
        back = t.cpu()                         # pageable D2H
        torch.cuda.synchronize()
        assert np.array_equal(back.numpy(), b)
        keep = b.copy()
        b[:] = 0
        b[:] = t.cpu().numpy()
        assert np.array_equal(b, keep)
        del t, back, b
    assert reused, "numpy never handed a freed registered page out again"
