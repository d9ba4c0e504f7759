"""CPU tests of the two oracle restatements (test infrastructure) and of their
pinning to the reference: the KAT, the committed goldens, and the property
tests of /root/reference/xrs_test.go ported with fixed seeds."""
import numpy as np
import pytest

from oracle.oracle_c import OracleError, OracleXRS
from oracle.xrs_oracle import XRS as PyXRS
from oracle.xrs_oracle import XRSError, gf_inv, gf_mul, make_xor_set, make_xor_set_old

ORACLES = [PyXRS, OracleXRS]
D, P = 12, 4


def encoded(x, rng, size, d=D, p=P):
    v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(d)]
    v += [np.zeros(size, np.uint8) for _ in range(p)]
    x.encode(v)
    return v


# ---------------------------------------------------------------- pinning
@pytest.mark.parametrize("cls", ORACLES)
def test_kat_5p5(cls):
    """xrs_test.go:102-122 TestXRS_Encode ("Powered by MATLAB")."""
    v = [np.array(a, np.uint8) for a in
         ([0, 0], [4, 7], [2, 4], [6, 9], [8, 11], [0, 0], [0, 0], [0, 0], [0, 0], [0, 0])]
    cls(5, 5).encode(v)
    exp = [[0, 0], [4, 7], [2, 4], [6, 9], [8, 11], [97, 156], [173, 117], [218, 110], [107, 59],
           [110, 153]]
    assert [list(map(int, a)) for a in v] == exp


def test_kat_rs_intermediate():
    """RS-form parity before piggyback for the 5+5 KAT."""
    x = PyXRS(5, 5)
    v = [np.array(a, np.uint8) for a in ([0, 0], [4, 7], [2, 4], [6, 9], [8, 11])]
    v += [np.zeros(2, np.uint8) for _ in range(5)]
    x.rs_encode(v)
    assert [list(map(int, a)) for a in v[5:]] == [[97, 156], [173, 125], [218, 106], [107, 57],
                                                  [110, 159]]


def test_gf_field():
    assert gf_mul(2, 0x80) == 0x1D  # x^8 = x^4+x^3+x^2+1 (0x11d)
    for a in range(1, 256):
        assert gf_mul(a, gf_inv(a)) == 1


def test_generator_12p4():
    g = PyXRS(12, 4).gen
    assert bytes(g[12]).hex() == "3daa5d96ad9ddd9847a77aba"
    assert bytes(g[15]).hex() == "965daa3d98dd9dadba7aa747"
    assert np.array_equal(g[:12], np.eye(12, dtype=np.uint8))


@pytest.mark.parametrize("S", [2, 64, 1026, 4096])
def test_golden_against_oracles(golden, S):
    for cls in ORACLES:
        x = cls(D, P)
        v = [r.copy() for r in golden[f"enc_S{S}_in"]] + [np.zeros(S, np.uint8) for _ in range(P)]
        x.encode(v)
        assert np.array_equal(np.stack(v), golden[f"enc_S{S}_out"])
        i = 0
        while f"rc{i}_S{S}_has" in golden:
            has = list(golden[f"rc{i}_S{S}_has"])
            need = list(golden[f"rc{i}_S{S}_need"])
            v = [r.copy() for r in golden[f"rc{i}_S{S}_in"]]
            x.reconst(v, has, need)
            assert np.array_equal(np.stack(v), golden[f"rc{i}_S{S}_out"]), (cls, i)
            i += 1


# ----------------------------------------------------------- structural
def test_make_xor_set_matches_old():
    """xrs_test.go:51-80 TestMakeXORSet (all d, p with d+p <= 256)."""
    for d in range(1, 256):
        for p in range(2, 257 - d):
            assert make_xor_set(d, p) == make_xor_set_old(d, p), (d, p)


def test_get_need_vects_all_configs():
    """xrs_test.go:124-156 TestXRS_GetNeedVects, on the numpy oracle (a subset of
    p per d keeps it fast; the product library runs the full sweep)."""
    for d in range(1, 256):
        for p in sorted({2, 3, 4, 5, 8, 16, 256 - d}):
            if p < 2 or d + p > 256:
                continue
            x = PyXRS(d, p)
            for i in range(d):
                a, b = x.get_need_vects(i)
                assert b[0] == d
                assert sorted(a + [i]) == x.xor_set[b[1]]


def test_errors():
    with pytest.raises(XRSError, match="illegal parity"):
        PyXRS(4, 1)
    with pytest.raises(OracleError):
        OracleXRS(4, 1)
    x = PyXRS(12, 4)
    with pytest.raises(XRSError, match="vect size not even: 3"):
        x.encode([np.zeros(3, np.uint8)] * 16)
    with pytest.raises(XRSError, match="illegal data index: 12"):
        x.get_need_vects(12)


# ------------------------------------------------------ ported properties
@pytest.mark.parametrize("cls", ORACLES)
def test_reconst_one_need_set_only(cls, rng):
    """xrs_test.go:158-227 testReconstOne (S=2): every byte outside the need set
    is zeroed, so reads must stay inside it."""
    size = 2
    x = cls(D, P)
    for lost in range(D):
        exp = encoded(x, rng, size)
        res = [r.copy() for r in exp]
        res[lost][:] = 0
        a_need, b_need = x.get_need_vects(lost)
        half = size // 2
        for j in range(D + P):
            if j not in a_need:
                res[j][:half] = 0
        for j in range(D, D + P):
            if j not in b_need:
                res[j][half:] = 0
        x.reconst_one(res, lost)
        assert np.array_equal(res[lost], exp[lost]), lost


def test_retrieve_rs_involution(rng):
    """xrs_test.go:229-259 TestXRS_RetrieveRS."""
    for cls in ORACLES:
        x = cls(D, P)
        v = [rng.integers(0, 256, size=1024, dtype=np.uint8) for _ in range(D + P)]
        r = [a.copy() for a in v]
        x.retrieve_rs(r, list(rng.permutation(D + P)))
        x.retrieve_rs(r, list(rng.permutation(D + P)))
        assert all(np.array_equal(a, b) for a, b in zip(v, r))


def _lost_random(rng, n, k):
    return [int(v) for v in rng.permutation(n)[:k]]


@pytest.mark.parametrize("cls", ORACLES)
def test_reconst_random(cls, rng):
    """xrs_test.go:261-314 testReconst (12+4, S=1024, 128 loops)."""
    x = cls(D, P)
    size = 1024
    for _ in range(128):
        exp = encoded(x, rng, size)
        lost = _lost_random(rng, D + P, int(rng.integers(0, P + 1)))
        need = lost[:int(rng.integers(0, len(lost) + 1))]
        if len(need) == 1:
            lost = need
        has = [i for i in range(D + P) if i not in lost]
        act = [np.zeros(size, np.uint8) for _ in range(D + P)]
        for h in has:
            act[h][:] = exp[h]
        for n in need:
            if rng.integers(0, 4) == 0:
                act[n][:] = exp[n]
        x.reconst(act, has, need)
        for n in need:
            assert np.array_equal(act[n], exp[n])


@pytest.mark.parametrize("cls", ORACLES)
def test_update_equals_reencode(cls, rng):
    """xrs_test.go:316-359 testUpdate."""
    x = cls(D, P)
    size = 1024
    for row in range(D):
        act = encoded(x, rng, size)
        new = rng.integers(0, 256, size=size, dtype=np.uint8)
        x.update(act[row], new, row, act[D:])
        exp = [a.copy() for a in act]
        exp[row] = new
        x.encode(exp)
        for j in range(D, D + P):
            assert np.array_equal(act[j], exp[j])


@pytest.mark.parametrize("cls", ORACLES)
@pytest.mark.parametrize("to_zero", [True, False])
def test_replace_equals_reencode(cls, to_zero, rng):
    """xrs_test.go:361-421 testReplace (fewer loops; the GPU test runs 1024)."""
    x = cls(D, P)
    size = 1024
    for _ in range(64):
        n = int(rng.integers(0, D + 1))
        rows = [int(v) for v in rng.permutation(D)[:n]] or [0]
        full = encoded(x, rng, size)
        data = [full[r].copy() for r in rows]
        zeroed = [a.copy() for a in full]
        for r in rows:
            zeroed[r][:] = 0
        x.encode(zeroed)
        act = [a.copy() for a in (full if to_zero else zeroed)]
        exp = zeroed if to_zero else full
        x.replace(data, rows, act[D:])
        for j in range(D, D + P):
            assert np.array_equal(act[j], exp[j])


def test_c_vs_numpy_other_configs(rng):
    """Cross-check the two restatements on non-headline (d, p)."""
    for d, p in [(1, 2), (2, 3), (5, 5), (10, 4), (6, 3), (20, 8), (3, 9)]:
        xc, xp = OracleXRS(d, p), PyXRS(d, p)
        for size in (2, 34, 514):
            v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(d)]
            v += [np.zeros(size, np.uint8) for _ in range(p)]
            vc = [a.copy() for a in v]
            xc.encode(vc)
            xp.encode(v)
            assert all(np.array_equal(a, b) for a, b in zip(v, vc))
            lost = _lost_random(rng, d + p, p)
            need = lost[: max(1, len(lost) - 1)]
            has = [i for i in range(d + p) if i not in lost]
            a1 = [a.copy() for a in v]
            a2 = [a.copy() for a in v]
            xc.reconst(a1, has, need)
            xp.reconst(a2, has, need)
            assert all(np.array_equal(a, b) for a, b in zip(a1, a2))


# ------------------------------------------------ CPU baseline (batch) paths
@pytest.mark.parametrize("level", ["scalar", "avx2", "native"])
@pytest.mark.parametrize("d,p", [(12, 4), (5, 5), (20, 3)])
def test_cpu_baseline_batch_paths(monkeypatch, level, d, p):
    """The timed CPU baseline (oxrs_encode_batch / oxrs_reconst_one_batch, at
    every SIMD level: scalar, AVX2, and the CPU's widest, AVX-512BW here) equals
    the per-stripe restatement, on ragged sizes and several threads.  The GPU
    tests use the batch path as their reference, so it is pinned here."""
    from oracle.oracle_c import lib
    if level == "avx2" and lib().oxrs_simd_level() < 1:
        pytest.skip("no AVX2")
    if level != "native":
        monkeypatch.setenv("OXRS_SIMD", level)
    rng = np.random.default_rng(11)
    o = OracleXRS(d, p)
    for size, n, threads in ((2, 3, 1), (34, 5, 2), (4096, 7, 3), (40000, 3, 2), (65602, 2, 1)):
        host = rng.integers(0, 256, size=(n, d + p, size), dtype=np.uint8)
        ref = host.copy()
        for s in range(n):
            v = [ref[s, i] for i in range(d + p)]
            o.encode(v)
        o.encode_batch(host, size, n, threads)
        assert np.array_equal(host, ref), (level, size)
        k = int(rng.integers(0, d))
        host[:, k] = 0x5A
        o.reconst_one_batch(host, size, n, k, threads)
        assert np.array_equal(host, ref), (level, size, k)


@pytest.mark.parametrize("level", ["scalar", "avx2", "native"])
@pytest.mark.parametrize("d,p", [(12, 4), (5, 5), (20, 3)])
def test_cpu_baseline_update_replace_batch(monkeypatch, level, d, p):
    """The config-4 CPU baseline (oxrs_update_batch / oxrs_replace_batch, the
    reference's two passes per op, xrs.go:324-387) equals the per-stripe
    restatement (oxrs_update / oxrs_replace) at every SIMD level."""
    from oracle.oracle_c import lib
    if level == "avx2" and lib().oxrs_simd_level() < 1:
        pytest.skip("no AVX2")
    if level != "native":
        monkeypatch.setenv("OXRS_SIMD", level)
    rng = np.random.default_rng(12)
    o = OracleXRS(d, p)
    for size, n, threads in ((2, 3, 1), (34, 5, 2), (4096, 7, 3), (40000, 3, 2), (65602, 2, 1)):
        row = int(rng.integers(0, d))
        host = rng.integers(0, 256, size=(n, 2 + p, size), dtype=np.uint8)
        ref = host.copy()
        for s in range(n):
            o.update(ref[s, 0], ref[s, 1], row, [ref[s, 2 + r] for r in range(p)])
        o.update_batch(host, size, n, row, threads)
        assert np.array_equal(host, ref), ("update", level, size)
        rows = [int(r) for r in rng.choice(d, size=min(4, d), replace=False)]
        host = rng.integers(0, 256, size=(n, len(rows) + p, size), dtype=np.uint8)
        ref = host.copy()
        for s in range(n):
            o.replace([ref[s, i] for i in range(len(rows))], rows,
                      [ref[s, len(rows) + r] for r in range(p)])
        o.replace_batch(host, size, n, rows, threads)
        assert np.array_equal(host, ref), ("replace", level, size)


@pytest.mark.parametrize("cls", ORACLES)
@pytest.mark.parametrize("S", [34, 2048])
@pytest.mark.parametrize("d,p", [(10, 4), (6, 3), (5, 5), (4, 2), (20, 4), (1, 2), (30, 6)])
def test_golden_codecs(golden_codecs, cls, d, p, S):
    """Both restatements reproduce the committed goldens of the other codecs
    (tests/golden/make_golden_codecs.py): Encode, Reconst, Update, Replace."""
    g, k, x = golden_codecs, f"d{d}p{p}_S{S}_", cls(d, p)
    v = [r.copy() for r in g[k + "enc_in"]] + [np.zeros(S, np.uint8) for _ in range(p)]
    x.encode(v)
    assert np.array_equal(np.stack(v), g[k + "enc_out"])
    for i in range(2):
        v = [r.copy() for r in g[k + f"rc{i}_in"]]
        x.reconst(v, list(g[k + f"rc{i}_has"]), list(g[k + f"rc{i}_need"]))
        assert np.array_equal(np.stack(v), g[k + f"rc{i}_out"]), i
    par = [r.copy() for r in g[k + "up_in"]]
    x.update(g[k + "up_old"].copy(), g[k + "up_new"].copy(), int(g[k + "up_row"][0]), par)
    assert np.array_equal(np.stack(par), g[k + "up_out"])
    par = [r.copy() for r in g[k + "rp_in"]]
    x.replace([r.copy() for r in g[k + "rp_data"]], list(g[k + "rp_rows"]), par)
    assert np.array_equal(np.stack(par), g[k + "rp_out"])
