"""Which kernel each launch runs (xrs_trace_kernels), on full-chip grids:
the shapes DESIGN.md §4 names for the bench launches and the staged Reconst
patterns, each result also checked against the oracle.  Reference semantics:
xrs.go:103-128 (Encode), :175-221 (ReconstOne), :236-320 (Reconst)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import xrs_amd  # noqa: E402
from oracle.oracle_c import OracleXRS  # noqa: E402

D, P = 12, 4


def _traced(fn):
    xrs_amd.trace_kernels(True)
    try:
        fn()
        torch.cuda.synchronize()
    finally:
        xrs_amd.trace_kernels(False)
    return list(xrs_amd.traced_kernels())


def test_library_is_this_tree():
    """The library these GPU tests load was built from this tree's sources:
    xrs_version() carries the source digest (xrs_amd/csrc/version.cpp), the
    tree's digest is recomputed here (xrs_amd.source_hash)."""
    built, tree = xrs_amd.library_source_hash(), xrs_amd.source_hash()
    print(f"library {xrs_amd.version()}, tree sources {tree}")
    assert built == tree, f"stale library: built from {built}, tree is {tree}"


@pytest.fixture(scope="module")
def codec():
    return xrs_amd.XRS(D, P), OracleXRS(D, P)


@pytest.mark.parametrize("size,n,enc,rec", [
    (4096, 1024, "enc_ws_kernel<12, 256>",
     "rows_kernel<2, 12, 4, false, true, 256>"),
    (1 << 20, 8, "pair_kernel<4, 12, false, true, 128, true>",
     "rows_kernel<2, 12, 4, false, true, 1024>"),
])
def test_headline_shapes(codec, size, n, enc, rec):
    x, o = codec
    rng = np.random.Generator(np.random.PCG64(11))
    host = rng.integers(0, 256, size=(n, D + P, size), dtype=np.uint8)
    t = torch.from_numpy(host).cuda()
    s = torch.cuda.current_stream().cuda_stream
    assert _traced(lambda: x.encode_batched(t.data_ptr(), size, size, (D + P) * size, n, s)) == [enc]
    ref = host.copy()
    o.encode_batch(ref, size, n)
    assert np.array_equal(t.cpu().numpy(), ref)
    t[:, 3].zero_()
    assert _traced(lambda: x.reconst_one_batched(t.data_ptr(), size, size, (D + P) * size, n, 3,
                                                 s)) == [rec]
    assert np.array_equal(t.cpu().numpy(), ref)


# (lost = needed, every survivor in dpHas) -> the staged kernel that runs
STAGED = [
    ([2, 9], 4096, "staged_ws_kernel<12, 14, 2, 2, 256, 1>"),
    ([0, 1, 2], 4096, "staged_ws_kernel<12, 13, 3, 3, 256, 1>"),
    ([12], 4096, "staged_ws_kernel<12, 15, 1, 1, 256, 1>"),
    ([13], 4096, "staged_ws_kernel<12, 14, 1, 1, 256, 1>"),
    ([15], 1 << 20, "staged_ws_kernel<12, 14, 1, 1, 512, 1>"),
    ([12], 1 << 20, "staged_ws_kernel<12, 15, 1, 1, 512, 1>"),
    ([0, 13], 4096, "staged_ws_kernel<12, 14, 2, 2, 256, 1>"),
    ([0, 5], 1 << 20, "staged_wsp_kernel<12, 14, 2, 2, 512>"),  # 16 stripes: 4 tiles per CU, the gate
    ([0, 6], 1 << 20, "staged_ws_kernel<12, 14, 2, 2, 512, 1>"),  # 8 stripes: 2 tiles per CU, under it
    ([0, 5, 7], 1 << 20, "staged_ws_kernel<12, 13, 3, 3, 256, 1>"),
]


@pytest.mark.parametrize("lost,size,kernel", STAGED)
def test_staged_patterns(codec, lost, size, kernel):
    x, o = codec
    n = 1024 if size == 4096 else 16 if kernel.startswith("staged_wsp") else 8
    rng = np.random.Generator(np.random.PCG64(12))
    host = rng.integers(0, 256, size=(n, D + P, size), dtype=np.uint8)
    o.encode_batch(host, size, n)
    host[:, lost] = 0xC3
    has = [i for i in range(D + P) if i not in lost]
    t = torch.from_numpy(host).cuda()
    s = torch.cuda.current_stream().cuda_stream
    got = _traced(lambda: x.reconst_batched(t.data_ptr(), size, size, (D + P) * size, n, has,
                                            lost, s))
    assert got == [kernel], got
    out = t.cpu().numpy()
    for st in (0, n // 2, n - 1):
        w = [host[st, i].copy() for i in range(D + P)]
        o.reconst(w, has, lost)
        assert np.array_equal(out[st], np.stack(w)), (lost, st)
