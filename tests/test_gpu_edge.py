"""GPU edge cases of general Reconst (xrs.go:236-301) against the oracle:
repeated indexes (the reference's loops apply an XOR once per occurrence),
a need list holding survivors, losses with an empty need (side effects only),
and error ordering."""
import numpy as np
import pytest

import xrs_amd
from oracle.oracle_c import OracleError, OracleXRS

pytestmark = pytest.mark.gpu
D, P = 12, 4


def stripe(rng, size):
    o = OracleXRS(D, P)
    v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(D)]
    v += [np.zeros(size, np.uint8) for _ in range(P)]
    o.encode(v)
    return v


CASES = [
    (list(range(2, 16)) + [14, 15], [0, 1]),          # repeated survivors (parity, twice)
    (list(range(2, 16)) + [13], [0, 1, 1]),            # repeated need
    (list(range(1, 14)), [14, 14, 15, 0]),             # repeated parity need (re-piggyback x2)
    ([i for i in range(16) if i not in (3, 13)], [3, 13, 5]),  # need holds a survivor (5)
    ([i for i in range(16) if i not in (3, 13)], []),  # losses, nothing needed: side effects
    (list(range(16)), [14]),                           # nothing lost, parity "needed"
    (list(range(4, 16)), [0, 1, 2, 3]),                # exactly d survivors
]


@pytest.mark.parametrize("has,need", CASES)
@pytest.mark.parametrize("size", [2, 4096, 1030])
def test_reconst_edge_vs_oracle(rng, has, need, size):
    v = stripe(rng, size)
    for i in range(D + P):
        if i not in has:
            v[i][:] = 0x5A
    a = [r.copy() for r in v]
    b = [r.copy() for r in v]
    xrs_amd.XRS(D, P).reconst(a, has, need)
    OracleXRS(D, P).reconst(b, has, need)
    for i in range(D + P):
        assert np.array_equal(a[i], b[i]), i


# Step-by-step plans that span more than one launch while a need row is also a
# GF source (dp_has[:d]): no launch may read a row an earlier launch of the
# plan wrote (codec.cpp step 3).
MULTI_LAUNCH = [
    (12, 4, list(range(0, 11)) + [13, 14, 15], [13, 0, 1, 2, 11]),  # > 4 needs, piggybacked survivor
    (12, 4, list(range(0, 11)) + [13, 14, 15], [0, 13, 1, 11, 2, 12, 14]),
    (12, 4, [i for i in range(16) if i not in (3, 7)], [3, 14, 13, 7, 5, 15]),
    (30, 4, list(range(30)), [29, 31]),                              # d > kMaxSrc, need holds a survivor
    (30, 4, [i for i in range(34) if i != 5], [5, 29, 32, 31, 0]),
    (28, 6, [i for i in range(34) if i not in (1, 2)], [1, 30, 2, 0, 31, 33]),
]


@pytest.mark.parametrize("d,p,has,need", MULTI_LAUNCH)
@pytest.mark.parametrize("size", [2, 4096, 1030])
def test_reconst_multi_launch_aliasing_vs_oracle(rng, d, p, has, need, size):
    o = OracleXRS(d, p)
    v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(d)]
    v += [np.zeros(size, np.uint8) for _ in range(p)]
    o.encode(v)
    for i in range(d + p):
        if i not in has:
            v[i][:] = 0x5A
    a = [r.copy() for r in v]
    b = [r.copy() for r in v]
    xrs_amd.XRS(d, p).reconst(a, has, need)
    o.reconst(b, has, need)
    for i in range(d + p):
        assert np.array_equal(a[i], b[i]), i


@pytest.mark.parametrize("has,need,msg", [
    (list(range(11)), [12, 13], "too few survivors"),
    (list(range(12)) + [16], [13, 14], "illegal index"),
    ([0] * 12 + [12], [13, 14], "singular matrix"),
    (list(range(16)), [-1], "illegal data index: -1"),
])
def test_reconst_errors_match_oracle(rng, has, need, msg):
    v = stripe(rng, 64)
    for i in range(D + P):
        if i not in has:
            v[i][:] = 0
    a = [r.copy() for r in v]
    b = [r.copy() for r in v]
    with pytest.raises(xrs_amd.XRSError, match=msg):
        xrs_amd.XRS(D, P).reconst(a, has, need)
    with pytest.raises(OracleError):
        OracleXRS(D, P).reconst(b, has, need)
    for i in range(D + P):  # the same (possibly partial) side effects
        assert np.array_equal(a[i], b[i]), i


@pytest.mark.gpu
def test_cpp_port_under_host_asan():
    """The C++ port of xrs_test.go linked against an ASan/UBSan (host code
    only) build of the library sources: no host memory errors on GPU paths."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "cpp", "build", "xrs_test_asan")
    if not os.path.exists(exe):
        pytest.skip("ASan build not present (tools/build_asan.sh)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=900,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]


@pytest.fixture(params=["staged", "staged_early", "staged_late", "staged_late_rt", "stepwise"])
def reconst_mode(request, monkeypatch):
    monkeypatch.delenv("XRS_RECONST", raising=False)
    monkeypatch.delenv("XRS_STAGED_LATE", raising=False)
    monkeypatch.delenv("XRS_STAGED_CT", raising=False)
    if request.param == "staged_early":
        monkeypatch.setenv("XRS_STAGED_LATE", "0")
    elif request.param == "staged_late":  # compile-time kernel where it applies
        monkeypatch.setenv("XRS_STAGED_LATE", "1")
    elif request.param == "staged_late_rt":  # the runtime-count late kernel
        monkeypatch.setenv("XRS_STAGED_LATE", "1")
        monkeypatch.setenv("XRS_STAGED_CT", "0")
    elif request.param == "stepwise":
        monkeypatch.setenv("XRS_RECONST", "steps")
    return request.param


@pytest.mark.parametrize("size", [2, 4096, 1030])
def test_reconst_random_both_paths(rng, reconst_mode, size):
    """General Reconst through the staged one-pass kernel and the step-by-step
    plan: identical buffers (side effects included) to the oracle."""
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    for _ in range(60):
        v = stripe(rng, size)
        lost = [int(t) for t in rng.permutation(D + P)[: int(rng.integers(0, P + 1))]]
        need = lost[: int(rng.integers(0, len(lost) + 1))]
        if rng.integers(0, 5) == 0 and need:
            need = need + [need[0]]  # a repeated need
        has = [i for i in range(D + P) if i not in lost]
        if rng.integers(0, 4) == 0:
            has = list(rng.permutation(has))  # survivors in any order
        for t in lost:
            v[t][:] = rng.integers(0, 256, size=size, dtype=np.uint8)
        a = [r.copy() for r in v]
        b = [r.copy() for r in v]
        x.reconst(a, has, need)
        o.reconst(b, has, need)
        for i in range(D + P):
            assert np.array_equal(a[i], b[i]), (reconst_mode, lost, need, i)


@pytest.mark.parametrize("d,p", [(10, 4), (6, 3), (4, 2), (14, 2), (3, 9), (16, 4), (15, 5),
                                 (16, 6)])
def test_reconst_other_configs_both_paths(rng, reconst_mode, d, p):
    """Per-stripe Reconst on other codecs; 16+4 / 15+5 read more than 16
    b-rows (the wide wave-specialised kernel), 16+6 has five retrieveRS rows,
    and 1,030-B vects have a ragged end (both run the step plan)."""
    x, o = xrs_amd.XRS(d, p), OracleXRS(d, p)
    for it in range(20):
        size = 1030 if it % 4 == 3 else 1024
        v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(d)]
        v += [np.zeros(size, np.uint8) for _ in range(p)]
        o.encode(v)
        lost = [int(t) for t in rng.permutation(d + p)[: int(rng.integers(1, p + 1))]]
        need = lost[: int(rng.integers(0, len(lost) + 1))]
        has = [i for i in range(d + p) if i not in lost]
        a = [r.copy() for r in v]
        b = [r.copy() for r in v]
        x.reconst(a, has, need)
        o.reconst(b, has, need)
        for i in range(d + p):
            assert np.array_equal(a[i], b[i]), (reconst_mode, d, p, lost, need, i)


@pytest.mark.parametrize("order", ["sorted", "reversed"])
def test_reconst_every_loss_pattern(rng, reconst_mode, order):
    """Every loss set of 1..p shards of a 12+4 stripe (2,516 patterns), need =
    the lost set, survivors sorted or reversed (reversed makes the first d
    survivors parity-heavy, so the staged kernel reads extra a-rows): buffers
    identical to the oracle, side effects included."""
    from itertools import combinations
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    base = stripe(rng, 64)
    for k in range(1, P + 1):
        for lost in combinations(range(D + P), k):
            has = [i for i in range(D + P) if i not in lost]
            if order == "reversed":
                has = has[::-1]
            a = [r.copy() for r in base]
            for t in lost:
                a[t][:] = 0xA5
            b = [r.copy() for r in a]
            x.reconst(a, has, list(lost))
            o.reconst(b, has, list(lost))
            for i in range(D + P):
                assert np.array_equal(a[i], b[i]), (lost, order, i)


@pytest.mark.parametrize("ct", ["1", "0", "0_onewave", "early", "late", "ws128", "ws256", "ws512",
                                "ws128o5"])
@pytest.mark.parametrize("size,n", [(4096, 600), (1 << 20, 4), (4112, 520)])
def test_reconst_batched_full_grid_vs_oracle(rng, monkeypatch, ct, size, n):
    """General Reconst of batches large enough for the bandwidth kernels
    (compile-time staged kernel for lost data vects, XRS_STAGED_CT=0 the
    runtime-count one), side effects included, every stripe vs the oracle."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("XRS_STAGED_CT", "0" if ct.startswith("0") else "1")
    monkeypatch.delenv("XRS_STAGED_WS", raising=False)
    if ct == "0_onewave":  # the runtime-count one-wave late kernel
        monkeypatch.setenv("XRS_STAGED_WS", "0")
    if ct == "0":  # the runtime-count wave-specialised kernel
        monkeypatch.setenv("XRS_STAGED_WS", "rt")
    if ct in ("early", "late"):  # both phase layouts of the one-wave compile-time kernel
        monkeypatch.setenv("XRS_STAGED_EARLY", "1" if ct == "early" else "0")
        monkeypatch.setenv("XRS_STAGED_WS", "0")
    if ct.startswith("ws"):  # the wave-specialised kernel, T chunks per block
        monkeypatch.setenv("XRS_STAGED_WS", ct[2:])
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    host = rng.integers(0, 256, size=(n, D + P, size), dtype=np.uint8)
    o.encode_batch(host, size, n)
    s = torch.cuda.current_stream().cuda_stream
    for lost, need in (([0, 1], [0, 1]), ([0, 1, 2], [0, 1, 2]), ([0, 1, 2, 3], [0, 1, 2, 3]),
                       ([4, 9], [9, 4]), ([2, 5, 11], [5]), ([1, 13], [1, 13]), ([3, 7, 8], []),
                       ([12], [12]), ([14], [14])):
        h = host.copy()
        h[:, lost] = 0x5A
        has = [i for i in range(D + P) if i not in lost]
        t = torch.from_numpy(h).cuda()
        x.reconst_batched(t.data_ptr(), size, size, (D + P) * size, n, has, need, s)
        torch.cuda.synchronize()
        got = t.cpu().numpy()
        for st in range(n):
            w = [h[st, i].copy() for i in range(D + P)]
            o.reconst(w, has, need)
            assert np.array_equal(got[st], np.stack(w)), (lost, need, st)


@pytest.mark.parametrize("wsp,grid", [("512", ""), ("256", ""), ("512", "24"), ("256", "7"),
                                      ("512", "1"), ("", ""), ("", "13")])
@pytest.mark.parametrize("size,n", [(4096, 601), (1 << 20, 5)])
def test_reconst_batched_persistent_vs_oracle(rng, monkeypatch, wsp, grid, size, n):
    """The persistent wave-specialised kernel (staged_wsp_kernel; XRS_WSP
    forces it for 2-4 lost, the default runs it for 2 lost from 256 to 768
    KiB halves in launches of at least 4 tiles per CU, test_gpu_dispatch.py): every block takes several tiles from the launch's counter when
    XRS_WSP_GRID caps the grid (ragged last tile, uneven tile counts per
    block, both LDS slots reused), every stripe vs the oracle, side effects
    included (xrs.go:236-320)."""
    torch = pytest.importorskip("torch")
    if wsp:
        monkeypatch.setenv("XRS_WSP", wsp)
    else:  # the default: the persistent kernel only for large 2-lost launches
        monkeypatch.delenv("XRS_WSP", raising=False)
    monkeypatch.delenv("XRS_STAGED_WS", raising=False)
    monkeypatch.delenv("XRS_STAGED_CT", raising=False)
    if grid:
        monkeypatch.setenv("XRS_WSP_GRID", grid)
    else:
        monkeypatch.delenv("XRS_WSP_GRID", raising=False)
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    host = rng.integers(0, 256, size=(n, D + P, size), dtype=np.uint8)
    o.encode_batch(host, size, n)
    s = torch.cuda.current_stream().cuda_stream
    for lost, need in (([0, 1], [0, 1]), ([0, 1, 2], [0, 1, 2]), ([0, 1, 2, 3], [0, 1, 2, 3]),
                       ([4, 9], [9, 4]), ([2, 5, 11], [5])):
        h = host.copy()
        h[:, lost] = 0x5A
        has = [i for i in range(D + P) if i not in lost]
        t = torch.from_numpy(h).cuda()
        xrs_amd.trace_kernels(True)
        try:
            x.reconst_batched(t.data_ptr(), size, size, (D + P) * size, n, has, need, s)
            torch.cuda.synchronize()
        finally:
            xrs_amd.trace_kernels(False)
        names = list(xrs_amd.traced_kernels())
        persistent = [k for k in names if k.startswith("staged_wsp_kernel<12, ")]
        if sorted(lost) == sorted(need) and wsp:
            assert len(names) == 1 and persistent, names
        elif not wsp:  # these batches are under the default's size threshold
            assert not persistent, names
        got = t.cpu().numpy()
        for st in range(n):
            w = [h[st, i].copy() for i in range(D + P)]
            o.reconst(w, has, need)
            assert np.array_equal(got[st], np.stack(w)), (lost, need, st)


def test_reconst_persistent_concurrent_streams(rng, monkeypatch):
    """Persistent 2-lost launches on four streams at once (each launch owns
    its tile counter): every stripe of every batch vs the oracle."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("XRS_WSP", "512")
    monkeypatch.setenv("XRS_WSP_GRID", "64")  # many tiles per block, long overlap
    size, n = 1 << 20, 6
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    host = rng.integers(0, 256, size=(n, D + P, size), dtype=np.uint8)
    o.encode_batch(host, size, n)
    lost = [3, 8]
    h = host.copy()
    h[:, lost] = 0x5A
    has = [i for i in range(D + P) if i not in lost]
    streams = [torch.cuda.Stream() for _ in range(4)]
    ts = [torch.from_numpy(h).cuda() for _ in streams]
    torch.cuda.synchronize()
    xrs_amd.trace_kernels(True)
    try:
        for t, st in zip(ts, streams):
            x.reconst_batched(t.data_ptr(), size, size, (D + P) * size, n, has, lost, st.cuda_stream)
        torch.cuda.synchronize()
    finally:
        xrs_amd.trace_kernels(False)
    assert list(xrs_amd.traced_kernels()) == ["staged_wsp_kernel<12, 14, 2, 2, 512>"]
    want = []
    for st in range(n):
        w = [h[st, i].copy() for i in range(D + P)]
        o.reconst(w, has, lost)
        want.append(np.stack(w))
    for t in ts:
        got = t.cpu().numpy()
        for st in range(n):
            assert np.array_equal(got[st], want[st]), st


def test_reconst_persistent_counter_slots_reused(rng, monkeypatch):
    """320 persistent launches, 80 on each of four streams in two waves of at
    most 160 in flight, more than the 256 tile-counter slots of the device's
    ring (kernels.hip tile_counters): each launch's last block resets its
    slot, so every launch runs the persistent kernel (none falls back for want
    of a free slot) and every
    buffer equals the oracle after the same 80 calls (a repeated Reconst
    toggles the retrieveRS side effect, xrs.go:305-320, so the oracle replays
    every call)."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("XRS_WSP", "512")
    monkeypatch.setenv("XRS_WSP_GRID", "8")
    # a 20-block grid would take the latency-bound all-loads-first kernel;
    # XRS_STAGED_LATE=1 keeps it on the bandwidth path XRS_WSP forces
    monkeypatch.setenv("XRS_STAGED_LATE", "1")
    size, n, calls = 4096, 40, 80
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    host = rng.integers(0, 256, size=(n, D + P, size), dtype=np.uint8)
    o.encode_batch(host, size, n)
    lost = [2, 7]
    h = host.copy()
    h[:, lost] = 0x5A
    has = [i for i in range(D + P) if i not in lost]
    streams = [torch.cuda.Stream() for _ in range(4)]
    ts = [torch.from_numpy(h).cuda() for _ in streams]
    torch.cuda.synchronize()
    xrs_amd.trace_kernels(True)
    try:
        for c in range(calls):
            for t, st in zip(ts, streams):
                x.reconst_batched(t.data_ptr(), size, size, (D + P) * size, n, has, lost,
                                  st.cuda_stream)
            if c % 40 == 39:  # at most 160 launches queued: the slots are reused,
                torch.cuda.synchronize()  # never all held at once
    finally:
        xrs_amd.trace_kernels(False)
    assert xrs_amd.traced_kernels() == {"staged_wsp_kernel<12, 14, 2, 2, 512>": 4 * calls}
    want = []
    for st in range(n):
        w = [h[st, i].copy() for i in range(D + P)]
        for _ in range(calls):
            o.reconst(w, has, lost)
        want.append(np.stack(w))
    for t in ts:
        got = t.cpu().numpy()
        for st in range(n):
            assert np.array_equal(got[st], want[st]), st


@pytest.mark.parametrize("ws", ["", "0", "rt"])
@pytest.mark.parametrize("d,p", [(10, 4), (16, 4), (6, 3), (12, 4), (15, 5), (8, 4), (14, 4),
                                 (10, 2)])
@pytest.mark.parametrize("size,n", [(4096, 520), (1 << 20, 4)])
def test_reconst_batched_runtime_shapes_vs_oracle(rng, monkeypatch, ws, d, p, size, n):
    """General Reconst on full grids through the runtime-count staged kernels
    (default: wave-specialised for one lost parity; XRS_STAGED_WS=rt
    wave-specialised for every pattern, =0 the one-wave late kernel):
    other codecs and loss patterns with parity in them, side effects included,
    every stripe vs the oracle."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("XRS_STAGED_WS", ws)
    x, o = xrs_amd.XRS(d, p), OracleXRS(d, p)
    host = rng.integers(0, 256, size=(n, d + p, size), dtype=np.uint8)
    o.encode_batch(host, size, n)
    s = torch.cuda.current_stream().cuda_stream
    last = d + p - 1
    pats = [([0, 1], [0, 1]), ([0, 1, 2][:p], [0, 1, 2][:p]), ([d + 1], [d + 1]), ([d], [d]),
            ([0, d + 1], [0, d + 1]),
            ([1, 2, last], [1, 2, last]), ([0, 1, d, d + 1][:p], [0, 1, d, d + 1][:p]),
            ([3, d + 1], [3])]
    for lost, need in [pt for pt in pats if len(pt[0]) <= p]:  # at most p lost
        h = host.copy()
        h[:, lost] = 0xC3
        has = [i for i in range(d + p) if i not in lost]
        t = torch.from_numpy(h).cuda()
        x.reconst_batched(t.data_ptr(), size, size, (d + p) * size, n, has, need, s)
        torch.cuda.synchronize()
        got = t.cpu().numpy()
        for st in range(n):
            w = [h[st, i].copy() for i in range(d + p)]
            o.reconst(w, has, need)
            assert np.array_equal(got[st], np.stack(w)), (lost, need, st)


def test_codec_first_then_torch():
    """A codec call before torch touches the GPU, then torch: one HIP runtime,
    torch still sees the device, and a batched call on torch memory works."""
    import subprocess
    import sys
    code = """
import numpy as np, xrs_amd
x = xrs_amd.XRS(12, 4)
v = [np.full(4096, i, np.uint8) for i in range(16)]
x.encode(v)
import torch
assert torch.cuda.is_available()
assert len(xrs_amd.hip_runtimes()) == 1, xrs_amd.hip_runtimes()
t = torch.zeros(16 * 4096, dtype=torch.uint8, device="cuda")
for i in range(12):
    t[i * 4096:(i + 1) * 4096] = i
x.encode_batched(t.data_ptr(), 4096, 4096, 16 * 4096, 1, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
got = t.cpu().numpy().reshape(16, 4096)
for r in range(12, 16):
    assert np.array_equal(got[r], v[r]), r
print("ok")
"""
    import os
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
