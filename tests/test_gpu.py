"""GPU parity tests: the HIP path (through the C ABI) against the oracle, the
committed goldens and the reference's property tests (xrs_test.go), plus
size-independent round-trip properties at BASELINE.json's full sizes.

All tests run in ONE process on the GPU box (python -m pytest tests -m gpu)."""
import numpy as np
import pytest

import xrs_amd
from oracle.oracle_c import OracleXRS

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

D, P = 12, 4


@pytest.fixture(scope="module")
def cuda():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda:0")


def stream():
    return torch.cuda.current_stream().cuda_stream


def to_dev(a: np.ndarray, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def encoded_host(x, rng, size, d=D, p=P):
    v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(d)]
    v += [np.zeros(size, np.uint8) for _ in range(p)]
    x.encode(v)
    return v


# ============================================================ sync (host) API
def test_kat_5p5(cuda):
    """xrs_test.go:102-122 through the GPU path."""
    v = [np.array(a, np.uint8) for a in
         ([0, 0], [4, 7], [2, 4], [6, 9], [8, 11], [0, 0], [0, 0], [0, 0], [0, 0], [0, 0])]
    xrs_amd.XRS(5, 5).encode(v)
    assert [list(map(int, a)) for a in v[5:]] == [[97, 156], [173, 117], [218, 110], [107, 59],
                                                  [110, 153]]


@pytest.mark.parametrize("S", [2, 64, 1026, 4096])
def test_golden_sync(golden, cuda, S):
    x = xrs_amd.XRS(D, P)
    v = [r.copy() for r in golden[f"enc_S{S}_in"]] + [np.zeros(S, np.uint8) for _ in range(P)]
    x.encode(v)
    assert np.array_equal(np.stack(v), golden[f"enc_S{S}_out"])
    enc = golden[f"enc_S{S}_out"]
    i = 0
    while f"rc{i}_S{S}_has" in golden:
        v = [r.copy() for r in golden[f"rc{i}_S{S}_in"]]
        x.reconst(v, list(golden[f"rc{i}_S{S}_has"]), list(golden[f"rc{i}_S{S}_need"]))
        assert np.array_equal(np.stack(v), golden[f"rc{i}_S{S}_out"]), i
        i += 1
    for row in range(D):
        par = [r.copy() for r in enc[D:]]
        x.update(enc[row].copy(), golden[f"up_S{S}_row{row}_new"], row, par)
        assert np.array_equal(np.stack(par), golden[f"up_S{S}_row{row}_out"]), row
    for n in (1, 4, 12):
        for z in ("tozero", "fromzero"):
            rows = [int(r) for r in golden[f"rp_S{S}_n{n}_{z}_rows"]]
            par = [r.copy() for r in golden[f"rp_S{S}_n{n}_{z}_in"]]
            x.replace([enc[r].copy() for r in rows], rows, par)
            assert np.array_equal(np.stack(par), golden[f"rp_S{S}_n{n}_{z}_out"]), (n, z)


@pytest.mark.parametrize("size", [2, 4096, 1 << 20])
def test_reconst_one_need_set_only(cuda, rng, size):
    """xrs_test.go:158-227: bytes outside GetNeedVects are zeroed first."""
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    for lost in range(D):
        exp = encoded_host(o, rng, size)
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


def test_reconst_random_vs_oracle(cuda, rng):
    """xrs_test.go:261-314 testReconst (128 loops, S=1024); every buffer is
    compared with the oracle, so the side effects match too."""
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    size = 1024
    for _ in range(128):
        exp = encoded_host(o, rng, size)
        lost = [int(v) for v in rng.permutation(D + P)[: int(rng.integers(0, P + 1))]]
        need = lost[: int(rng.integers(0, len(lost) + 1))]
        if len(need) == 1:
            lost = need
        has = [i for i in range(D + P) if i not in lost]
        act = [np.zeros(size, np.uint8) for _ in range(D + P)]
        for h in has:
            act[h][:] = exp[h]
        for n in need:
            if rng.integers(0, 4) == 0:
                act[n][:] = exp[n]
        ref = [a.copy() for a in act]
        x.reconst(act, has, need)
        o.reconst(ref, has, need)
        for n in need:
            assert np.array_equal(act[n], exp[n])
        assert all(np.array_equal(a, b) for a, b in zip(act, ref))


def test_update_sync(cuda, rng):
    """xrs_test.go:316-359 testUpdate."""
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    for row in range(D):
        act = encoded_host(o, rng, 1024)
        new = rng.integers(0, 256, size=1024, dtype=np.uint8)
        x.update(act[row], new, row, act[D:])
        exp = [a.copy() for a in act]
        exp[row] = new
        o.encode(exp)
        assert all(np.array_equal(act[j], exp[j]) for j in range(D, D + P))


@pytest.mark.parametrize("to_zero", [True, False])
def test_replace_sync(cuda, rng, to_zero):
    """xrs_test.go:361-421 testReplace (1024 loops each direction)."""
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    size = 1024
    for _ in range(1024):
        n = int(rng.integers(0, D + 1))
        rows = [int(v) for v in rng.permutation(D)[:n]] or [0]
        full = encoded_host(o, rng, size)
        data = [full[r].copy() for r in rows]
        zeroed = [a.copy() for a in full]
        for r in rows:
            zeroed[r][:] = 0
        o.encode(zeroed)
        act = [a.copy() for a in (full if to_zero else zeroed)]
        exp = zeroed if to_zero else full
        x.replace(data, rows, act[D:])
        assert all(np.array_equal(act[j], exp[j]) for j in range(D, D + P))


@pytest.mark.parametrize("d,p", [(1, 2), (2, 3), (5, 5), (10, 4), (6, 3), (20, 8), (3, 9),
                                 (30, 6), (100, 10), (200, 56), (250, 6)])
def test_other_configs_sync(cuda, rng, d, p):
    """Runtime-shaped kernels, output groups (p > 4) and source chunks (d > 24)."""
    x, o = xrs_amd.XRS(d, p), OracleXRS(d, p)
    for size in (2, 34, 4096, 4114):
        v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(d)]
        v += [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(p)]  # garbage parity
        ref = [a.copy() for a in v]
        x.encode(v)
        o.encode(ref)
        assert all(np.array_equal(a, b) for a, b in zip(v, ref)), size
        for k in (0, d - 1):
            a = [r.copy() for r in v]
            a[k][:] = 0
            x.reconst_one(a, k)
            assert np.array_equal(a[k], v[k])
        lost = [int(t) for t in rng.permutation(d + p)[:p]]
        need = lost[: max(2, len(lost) - 1)]
        has = [i for i in range(d + p) if i not in lost]
        a1 = [r.copy() for r in v]
        a2 = [r.copy() for r in v]
        for t in lost:
            a1[t][:] = 0x5A
            a2[t][:] = 0x5A
        x.reconst(a1, has, need)
        o.reconst(a2, has, need)
        assert all(np.array_equal(a, b) for a, b in zip(a1, a2)), size
        row = int(rng.integers(0, d))
        new = rng.integers(0, 256, size=size, dtype=np.uint8)
        p1 = [r.copy() for r in v[d:]]
        p2 = [r.copy() for r in v[d:]]
        x.update(v[row], new, row, p1)
        o.update(v[row], new, row, p2)
        assert all(np.array_equal(a, b) for a, b in zip(p1, p2))
        rows = [int(t) for t in rng.permutation(d)[: max(1, d // 2)]]
        data = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in rows]
        x.replace(data, rows, p1)
        o.replace(data, rows, p2)
        assert all(np.array_equal(a, b) for a, b in zip(p1, p2))


@pytest.mark.parametrize("grouped", ["0", "1"])
@pytest.mark.parametrize("d,p", [(10, 4), (5, 5), (30, 6)])
def test_rows_runtime_loops(cuda, rng, monkeypatch, grouped, d, p):
    """Both loops of the runtime-count rows kernel (grouped loads: chosen for
    grids under one block per CU; one row at a time: larger grids), forced
    either way, on single stripes and on a batch: ReconstOne and the
    step-by-step Reconst plan, side effects included."""
    monkeypatch.setenv("XRS_ROWS_GROUPED", grouped)
    monkeypatch.setenv("XRS_RECONST", "steps")
    x, o = xrs_amd.XRS(d, p), OracleXRS(d, p)
    for size in (34, 4096):
        v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(d + p)]
        o.encode(v)
        a = [r.copy() for r in v]
        a[1][:] = 0
        x.reconst_one(a, 1)
        assert np.array_equal(a[1], v[1])
        lost = [int(t) for t in rng.permutation(d + p)[:p]]
        has = [i for i in range(d + p) if i not in lost]
        a1, a2 = [r.copy() for r in v], [r.copy() for r in v]
        x.reconst(a1, has, lost)
        o.reconst(a2, has, lost)
        assert all(np.array_equal(s, t) for s, t in zip(a1, a2)), size
    size, n = 4096, 300
    host = rng.integers(0, 256, size=(n, d + p, size), dtype=np.uint8)
    o.encode_batch(host, size, n)
    t = torch.from_numpy(host).cuda()
    t[:, 2].zero_()
    s = torch.cuda.current_stream().cuda_stream
    x.reconst_one_batched(t.data_ptr(), size, size, (d + p) * size, n, 2, s)
    torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy(), host)


def test_errors_on_gpu(cuda):
    x = xrs_amd.XRS(D, P)
    with pytest.raises(xrs_amd.XRSError, match="^vect size not even: 9$"):
        x.encode([np.zeros(9, np.uint8) for _ in range(16)])
    with pytest.raises(xrs_amd.XRSError, match="^illegal data index: -1$"):
        x.reconst([np.zeros(8, np.uint8) for _ in range(16)], list(range(16)), [-1])
    v = [np.zeros(8, np.uint8) for _ in range(16)]
    with pytest.raises(xrs_amd.XRSError, match="too few survivors"):
        x.reconst(v, list(range(11)), [12, 13])
    x.encode([np.zeros(0, np.uint8) for _ in range(16)])  # empty vects: no-op


# ============================================================ batched device API
def batch(rng, n, size, d=D, p=P):
    return rng.integers(0, 256, size=(n, d + p, size), dtype=np.uint8)


def oracle_encode_batch(o, host):
    h = host.copy()
    n, _, size = h.shape
    o.encode_batch(h, size, n)
    return h


# 1 MiB and 1 MiB + 2: the 12+4 Encode from 512 KiB halves runs the
# plain-order kernel specialization (pair_kernel<4, 12, false, true, 128, true>);
# aligned halves up to 128 KiB the wave-specialised enc_ws_kernel<12, 256>
# (XRS_ENC_WS=0: the pair kernel there too; =128 / 512: other block sizes;
# any other value, e.g. 1 or "on", forces it on at 256 chunks per block,
# 1 MiB included).
@pytest.mark.parametrize("enc_ws", ["", "0", "128", "512", "1", "on"])
@pytest.mark.parametrize("size", [4096, 2, 1026, 4112, 4128, 65536, 262144, 1 << 20, (1 << 20) + 2])
def test_encode_batched_vs_oracle(cuda, rng, monkeypatch, size, enc_ws):
    if enc_ws:
        monkeypatch.setenv("XRS_ENC_WS", enc_ws)
    else:
        monkeypatch.delenv("XRS_ENC_WS", raising=False)
    n = max(3, (8 << 20) // (16 * size))
    host = batch(rng, n, size)
    t = to_dev(host, cuda)
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    x.encode_batched(t.data_ptr(), size, size, 16 * size, n, stream())
    torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy(), oracle_encode_batch(o, host))


def test_encode_batched_padded_layout(cuda, rng):
    """Shard and stripe strides larger than the vect (and not 16-aligned)."""
    size, n = 4096, 37
    for shard_stride, stripe_stride in [(4096 + 16, 16 * (4096 + 16) + 64), (4099, 16 * 4099 + 5)]:
        buf = rng.integers(0, 256, size=n * stripe_stride, dtype=np.uint8)
        t = to_dev(buf, cuda)
        xrs_amd.XRS(D, P).encode_batched(t.data_ptr(), size, shard_stride, stripe_stride, n,
                                         stream())
        torch.cuda.synchronize()
        got = t.cpu().numpy()
        o = OracleXRS(D, P)
        for s in range(n):
            v = [buf[s * stripe_stride + i * shard_stride:][:size].copy() for i in range(D + P)]
            o.encode(v)
            for i in range(D + P):
                off = s * stripe_stride + i * shard_stride
                assert np.array_equal(got[off:off + size], v[i]), (s, i)
        # bytes between shards untouched
        mask = np.ones(len(buf), bool)
        for s in range(n):
            for i in range(D + P):
                off = s * stripe_stride + i * shard_stride
                mask[off:off + size] = False
        assert np.array_equal(got[mask], buf[mask])


@pytest.mark.parametrize("size", [4096, 1 << 20])
def test_reconst_one_batched_all_k(cuda, rng, size):
    n = 8 if size == 1 << 20 else 256
    o = OracleXRS(D, P)
    enc = oracle_encode_batch(o, batch(rng, n, size))
    x = xrs_amd.XRS(D, P)
    for k in range(D):
        a_need, b_need = x.get_need_vects(k)
        h = enc.copy()
        half = size // 2
        # garbage everywhere outside the need set
        for j in range(D + P):
            if j not in a_need:
                h[:, j, :half] = 0xA5
            if j != k and j < D or j in b_need:
                continue
            h[:, j, half:] = 0x3C
        h[:, k] = 0x77
        t = to_dev(h, cuda)
        x.reconst_one_batched(t.data_ptr(), size, size, 16 * size, n, k, stream())
        torch.cuda.synchronize()
        got = t.cpu().numpy()
        assert np.array_equal(got[:, k], enc[:, k]), k
        others = [j for j in range(D + P) if j != k]
        assert np.array_equal(got[:, others], h[:, others]), k  # nothing else written


def test_reconst_batched_vs_oracle(cuda, rng):
    size, n = 4096, 64
    o = OracleXRS(D, P)
    enc = oracle_encode_batch(o, batch(rng, n, size))
    x = xrs_amd.XRS(D, P)
    for _ in range(24):
        lost = [int(v) for v in rng.permutation(D + P)[: int(rng.integers(0, P + 1))]]
        need = lost[: int(rng.integers(0, len(lost) + 1))]
        has = [i for i in range(D + P) if i not in lost]
        h = enc.copy()
        for t_ in lost:
            h[:, t_] = rng.integers(0, 256, size=(n, size), dtype=np.uint8)
        t = to_dev(h, cuda)
        x.reconst_batched(t.data_ptr(), size, size, 16 * size, n, has, need, stream())
        torch.cuda.synchronize()
        got = t.cpu().numpy()
        for s in range(n):
            v = [h[s, i].copy() for i in range(D + P)]
            o.reconst(v, has, need)
            assert np.array_equal(got[s], np.stack(v)), (lost, need, s)


def test_update_replace_batched_vs_oracle(cuda, rng):
    size, n = 8 << 20, 4
    o = OracleXRS(D, P)
    enc = oracle_encode_batch(o, batch(rng, n, size))
    x = xrs_amd.XRS(D, P)
    new = rng.integers(0, 256, size=(n, size), dtype=np.uint8)
    row = 5
    t = to_dev(enc, cuda)
    tn = to_dev(new, cuda)
    S = 16 * size
    x.update_batched(t.data_ptr() + row * size, S, tn.data_ptr(), size, size, row,
                     t.data_ptr() + D * size, size, S, n, stream())
    torch.cuda.synchronize()
    got = t.cpu().numpy()
    for s in range(n):
        par = [enc[s, D + r].copy() for r in range(P)]
        o.update(enc[s, row], new[s], row, par)
        assert np.array_equal(got[s, D:], np.stack(par))
    # Replace(rows 0..3) from zero: parity of a stripe with rows 0..3 zeroed
    rows = [0, 1, 2, 3]
    z = enc.copy()
    z[:, rows] = 0
    z = oracle_encode_batch(o, z)
    t = to_dev(z, cuda)
    data = to_dev(np.ascontiguousarray(enc[:, rows]), cuda)
    x.replace_batched(data.data_ptr(), size, 4 * size, rows, size, t.data_ptr() + D * size, size,
                      S, n, stream())
    torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy()[:, D:], enc[:, D:])


# ============================================================ full-size properties
def _dev_random(n_bytes, dev, seed):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    return torch.randint(0, 256, (n_bytes,), dtype=torch.uint8, device=dev, generator=g)


@pytest.mark.parametrize("size,n", [(4096, 65536), (1 << 20, 512)])
def test_full_size_encode_erase_reconst(cuda, size, n):
    """BASELINE configs 2 and 3 at full size (4 GiB / 8 GiB): encode on the GPU,
    sample stripes against the oracle, then erase data shard k of EVERY stripe
    and ReconstOne it back (round trip, bit-exact on all stripes)."""
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    S = 16 * size
    t = _dev_random(n * S, cuda, 1234)
    x.encode_batched(t.data_ptr(), size, size, S, n, stream())
    torch.cuda.synchronize()
    v = t.view(n, 16, size)
    for s in (0, 1, n // 2, n - 1):
        host = v[s].cpu().numpy().copy()
        ref = [host[i].copy() for i in range(16)]
        o.encode(ref)
        assert np.array_equal(host, np.stack(ref)), s
    for k in (0, 7, 11):
        keep = v[:, k].clone()
        v[:, k].fill_(0)
        x.reconst_one_batched(t.data_ptr(), size, size, S, n, k, stream())
        torch.cuda.synchronize()
        assert torch.equal(v[:, k], keep), k
    # multi-loss: 2 data + 1 parity lost, rebuild all three
    lost = [3, 9, 14]
    keep = v[:, lost].clone()
    v[:, lost] = 0
    has = [i for i in range(16) if i not in lost]
    x.reconst_batched(t.data_ptr(), size, size, S, n, has, lost, stream())
    torch.cuda.synchronize()
    assert torch.equal(v[:, lost], keep)
    del t, v, keep
    torch.cuda.empty_cache()


@pytest.mark.parametrize("size,n", [(4096, 65536), (1 << 20, 512)])
def test_full_size_multi_loss_side_effects(cuda, size, n):
    """General Reconst (xrs.go:236-301) on full-size batches (4 / 8 GiB), the
    loss patterns of the reference's Reconst benchmark (lost data[:i]) and
    mixed data + parity losses, need = lost.  Without an oracle at this
    size, the expected buffers follow from the reference's semantics: every
    lost vect comes back whole, and every surviving piggybacked parity h
    leaves in RS form, b(h) = original b(h) ^ XOR of XORSet(h)'s a-halves
    (retrieveRS, xrs.go:305-320); everything else is unchanged."""
    x = xrs_amd.XRS(D, P)
    xs = x.xor_set
    S, H = 16 * size, size // 2
    t = _dev_random(n * S, cuda, 4321)
    x.encode_batched(t.data_ptr(), size, size, S, n, stream())
    torch.cuda.synchronize()
    v = t.view(n, 16, size)
    orig = v.clone()
    for lost in ([0, 1], [0, 1, 2], [0, 1, 2, 3], [3, 9, 14], [5, 13]):
        v.copy_(orig)
        v[:, lost] = 0x5A
        has = [i for i in range(16) if i not in lost]
        x.reconst_batched(t.data_ptr(), size, size, S, n, has, lost, stream())
        torch.cuda.synchronize()
        exp = orig.clone()
        for h in has:
            if h > D and xs.get(h):
                piggy = orig[:, xs[h][0], :H].clone()
                for j in xs[h][1:]:
                    piggy ^= orig[:, j, :H]
                exp[:, h, H:] ^= piggy
        assert torch.equal(v, exp), lost
        del exp
    del t, v, orig
    torch.cuda.empty_cache()


def test_update_linearity_full_size(cuda):
    """BASELINE config 4 (8 MiB vects): Update then Update back is the identity,
    and Update equals re-encode on sampled stripes."""
    size, n = 8 << 20, 32
    x = xrs_amd.XRS(D, P)
    S = 16 * size
    t = _dev_random(n * S, cuda, 99)
    x.encode_batched(t.data_ptr(), size, size, S, n, stream())
    v = t.view(n, 16, size)
    par0 = v[:, D:].clone()
    new = _dev_random(n * size, cuda, 7).view(n, size)
    row = 6
    x.update_batched(v[:, row].data_ptr(), S, new.data_ptr(), size, size, row,
                     v[:, D].data_ptr(), size, S, n, stream())
    par1 = v[:, D:].clone()
    x.update_batched(new.data_ptr(), size, v[:, row].data_ptr(), S, size, row,
                     v[:, D].data_ptr(), size, S, n, stream())
    torch.cuda.synchronize()
    assert torch.equal(v[:, D:], par0)
    v[:, row] = new
    x.encode_batched(t.data_ptr(), size, size, S, n, stream())
    torch.cuda.synchronize()
    assert torch.equal(v[:, D:], par1)
    del t, v, par0, par1, new
    torch.cuda.empty_cache()


def test_config5_per_gpu_share_round_trip(cuda):
    """BASELINE config 5's per-GPU share at full size: 8,192 stripes of 12+4
    1 MiB vects (128 GiB) resident on one GPU.  Encode, check sampled stripes
    against the oracle, erase data shard k of every stripe and ReconstOne it
    back bit for bit."""
    size, n = 1 << 20, 8192
    S = 16 * size
    free, _ = torch.cuda.mem_get_info(cuda)
    if free < n * S + n * size + (8 << 30):
        pytest.skip("needs ~145 GiB of free HBM")
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    t = _dev_random(n * S, cuda, 5)
    x.encode_batched(t.data_ptr(), size, size, S, n, stream())
    torch.cuda.synchronize()
    v = t.view(n, 16, size)
    for s in (0, 4097, n - 1):
        host = v[s].cpu().numpy().copy()
        ref = [host[i].copy() for i in range(16)]
        o.encode(ref)
        assert np.array_equal(host, np.stack(ref)), s
    k = 10
    keep = v[:, k].clone()
    v[:, k].fill_(0)
    x.reconst_one_batched(t.data_ptr(), size, size, S, n, k, stream())
    torch.cuda.synchronize()
    assert torch.equal(v[:, k], keep)
    del t, v, keep
    torch.cuda.empty_cache()


@pytest.mark.parametrize("S", [34, 2048])
@pytest.mark.parametrize("d,p", [(10, 4), (6, 3), (5, 5), (4, 2), (20, 4), (1, 2), (30, 6)])
def test_golden_codecs_gpu(golden_codecs, cuda, d, p, S):
    """The GPU (sync API, and batched for Encode / Reconst) reproduces the
    committed goldens of the other codecs bit for bit."""
    g, k, x = golden_codecs, f"d{d}p{p}_S{S}_", xrs_amd.XRS(d, p)
    v = [r.copy() for r in g[k + "enc_in"]] + [np.zeros(S, np.uint8) for _ in range(p)]
    x.encode(v)
    assert np.array_equal(np.stack(v), g[k + "enc_out"])
    t = to_dev(np.stack(v[:d] + [np.full(S, 7, np.uint8)] * p), cuda)
    x.encode_batched(t.data_ptr(), S, S, (d + p) * S, 1, stream())
    torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy(), g[k + "enc_out"])
    for i in range(2):
        has, need = [int(j) for j in g[k + f"rc{i}_has"]], [int(j) for j in g[k + f"rc{i}_need"]]
        v = [r.copy() for r in g[k + f"rc{i}_in"]]
        x.reconst(v, has, need)
        assert np.array_equal(np.stack(v), g[k + f"rc{i}_out"]), i
        t = to_dev(g[k + f"rc{i}_in"], cuda)
        x.reconst_batched(t.data_ptr(), S, S, (d + p) * S, 1, has, need, stream())
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy(), g[k + f"rc{i}_out"]), i
    par = [r.copy() for r in g[k + "up_in"]]
    x.update(g[k + "up_old"].copy(), g[k + "up_new"].copy(), int(g[k + "up_row"][0]), par)
    assert np.array_equal(np.stack(par), g[k + "up_out"])
    par = [r.copy() for r in g[k + "rp_in"]]
    x.replace([r.copy() for r in g[k + "rp_data"]], [int(j) for j in g[k + "rp_rows"]], par)
    assert np.array_equal(np.stack(par), g[k + "rp_out"])


@pytest.mark.parametrize("tail", ["overlap", "launch"])
@pytest.mark.parametrize("size,n", [(4100, 300), (1048578, 3), (34, 500), (18, 200), (4126, 100),
                                    (4098, 100), (65538, 20)])
def test_ragged_sizes_encode_reconst_one_vs_oracle(cuda, rng, monkeypatch, tail, size, n):
    """Vect sizes whose half is not a multiple of 16 (xrs.go:130-136 accepts
    any even size).  "overlap": the 16-byte launch ends with one overlapping
    chunk per row (the default); "launch": the separate byte-granular tail
    launch (XRS_TAIL=launch).  Both against the oracle, bytes between
    shards untouched (padded layout, odd strides)."""
    if tail == "launch":
        monkeypatch.setenv("XRS_TAIL", "launch")
    o = OracleXRS(D, P)
    x = xrs_amd.XRS(D, P)
    for shard_stride in (size, size + 7):
        stripe_stride = 16 * shard_stride + 3
        buf = rng.integers(0, 256, size=n * stripe_stride, dtype=np.uint8)
        t = to_dev(buf, cuda)
        x.encode_batched(t.data_ptr(), size, shard_stride, stripe_stride, n, stream())
        torch.cuda.synchronize()
        got = t.cpu().numpy()
        ref = buf.copy()
        for s in range(n):
            v = [ref[s * stripe_stride + i * shard_stride:][:size].copy() for i in range(D + P)]
            o.encode(v)
            for i in range(D + P):
                off = s * stripe_stride + i * shard_stride
                ref[off:off + size] = v[i]
        assert np.array_equal(got, ref)  # shards encoded, gaps untouched
        for k in (0, 7, 11):
            h = ref.copy()
            for s in range(n):
                off = s * stripe_stride + k * shard_stride
                h[off:off + size] = 0x5A
            t = to_dev(h, cuda)
            x.reconst_one_batched(t.data_ptr(), size, shard_stride, stripe_stride, n, k, stream())
            torch.cuda.synchronize()
            assert np.array_equal(t.cpu().numpy(), ref), (shard_stride, k)


CT_CODECS = [(4, 2), (6, 3), (8, 4), (10, 4), (12, 3), (14, 4), (16, 4), (20, 4), (10, 2), (6, 2),
             (8, 3), (10, 3), (12, 2)]


@pytest.mark.parametrize("mode", ["ct", "dyn", "ws"])
@pytest.mark.parametrize("d,p", CT_CODECS)
def test_compile_time_shapes_batched_vs_oracle(cuda, rng, monkeypatch, mode, d, p):
    """The compile-time Encode (pair_kernel<p, d>; enc_ws_kernel<d, 256> for
    d+4 when XRS_ENC_WS forces it) and ReconstOne (rows_kernel<2, d,
    |XORSet(bi)|>) shapes of common codecs, and the runtime-count kernels they
    replace (XRS_ENCODE_DYN / XRS_ROWS_DYN), on batches against the oracle:
    every k, aligned and ragged sizes."""
    if mode == "dyn":
        monkeypatch.setenv("XRS_ENCODE_DYN", "1")
        monkeypatch.setenv("XRS_ROWS_DYN", "1")
    if mode == "ws":
        if p != 4:
            pytest.skip("the wave-specialised Encode is a d+4 shape")
        monkeypatch.setenv("XRS_ENC_WS", "256")
    x, o = xrs_amd.XRS(d, p), OracleXRS(d, p)
    for size, n in ((4096, 64), (4100, 33), (34, 50)):
        host = rng.integers(0, 256, size=(n, d + p, size), dtype=np.uint8)
        t = to_dev(host, cuda)
        x.encode_batched(t.data_ptr(), size, size, (d + p) * size, n, stream())
        ref = host.copy()
        o.encode_batch(ref, size, n)
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy(), ref), size
        for k in range(d):
            t = to_dev(ref, cuda)
            t[:, k] = 0x5A
            x.reconst_one_batched(t.data_ptr(), size, size, (d + p) * size, n, k, stream())
            torch.cuda.synchronize()
            assert np.array_equal(t.cpu().numpy(), ref), (size, k)


PAD_CODECS = [(11, 4), (13, 4), (9, 3), (7, 3), (18, 4), (5, 4), (15, 4), (9, 2)]


@pytest.mark.parametrize("mode", ["pad", "nopad"])
@pytest.mark.parametrize("d,p", PAD_CODECS)
def test_padded_shapes_batched_vs_oracle(cuda, rng, monkeypatch, mode, d, p):
    """Codecs without their own compile-time Encode / ReconstOne shape run
    the nearest larger instantiation with up to 3 padding rows (zero tables,
    no piggyback; kernels.hip pad_count); XRS_PAD=0 runs the runtime-count
    kernels.  Both against the oracle on full grids and ragged sizes, every
    k, and the trace names the padded instantiation."""
    if mode == "nopad":
        monkeypatch.setenv("XRS_PAD", "0")
    x, o = xrs_amd.XRS(d, p), OracleXRS(d, p)
    for size, n in ((4096, 520), (4100, 33), (1 << 20, 2)):
        host = rng.integers(0, 256, size=(n, d + p, size), dtype=np.uint8)
        t = to_dev(host, cuda)
        xrs_amd.trace_kernels(True)
        x.encode_batched(t.data_ptr(), size, size, (d + p) * size, n, stream())
        torch.cuda.synchronize()
        xrs_amd.trace_kernels(False)
        names = list(xrs_amd.traced_kernels())
        if size == 4096:  # compile-time counts (pair_kernel<p, C, ...>) vs runtime (-1);
            # padding applies to halves up to 4 KiB only
            assert (f"pair_kernel<{p}, -1," in names[0]) == (mode == "nopad"), names
        ref = host.copy()
        o.encode_batch(ref, size, n)
        assert np.array_equal(t.cpu().numpy(), ref), size
        for k in range(d):
            t = to_dev(ref, cuda)
            t[:, k] = 0x5A
            x.reconst_one_batched(t.data_ptr(), size, size, (d + p) * size, n, k, stream())
            torch.cuda.synchronize()
            assert np.array_equal(t.cpu().numpy(), ref), (size, k)


@pytest.mark.parametrize("mode", ["ct", "dyn"])
@pytest.mark.parametrize("size,n", [(4096, 40), (9000, 20), (8200, 9), (34, 30)])
def test_replace_batched_every_n_vs_oracle(cuda, rng, monkeypatch, mode, size, n):
    """Replace(n) for n = 1..8 at 12+4 (the reference's Replace benchmark
    rows, xrs_test.go:627-680): compile-time source counts (halves > 4 KiB,
    or n >= 5) and the runtime-count kernel (XRS_REPLACE_DYN), both
    directions of the reference's test (zero -> data, data -> zero)."""
    if mode == "dyn":
        monkeypatch.setenv("XRS_REPLACE_DYN", "1")
    x, o = xrs_amd.XRS(D, P), OracleXRS(D, P)
    for nrep in range(1, 9):
        rows = [int(v) for v in rng.permutation(D)[:nrep]]
        data = rng.integers(0, 256, size=(n, nrep, size), dtype=np.uint8)
        par = rng.integers(0, 256, size=(n, P, size), dtype=np.uint8)
        td, tp = to_dev(data, cuda), to_dev(par, cuda)
        x.replace_batched(td.data_ptr(), size, nrep * size, rows, size, tp.data_ptr(), size,
                          P * size, n, stream())
        torch.cuda.synchronize()
        ref = par.copy()
        for st in range(n):
            pv = [ref[st, q] for q in range(P)]
            o.replace([data[st, i].copy() for i in range(nrep)], rows, pv)
        assert np.array_equal(tp.cpu().numpy(), ref), (nrep, rows)


@pytest.mark.parametrize("d,p,size,n", [(12, 3, 4096, 24), (10, 4, 4096, 24), (13, 2, 4100, 24),
                                        (12, 3, 1 << 16, 24), (12, 4, 4096, 24), (12, 4, 4100, 600),
                                        (12, 4, 4098, 600), (12, 4, 1048578, 6)])
def test_recommended_layout_vs_oracle(cuda, rng, d, p, size, n):
    """The layout xrs_batch_layout recommends (a power-of-two stripe stride
    with a gap after the last shard when that costs <= 1/7; odd sizes shifted
    by the base offset that aligns the b-halves, codec.cpp): Encode, every
    ReconstOne and a 2-loss Reconst against the oracle, full-chip grids for
    the odd 12+4 sizes, with the gap and offset bytes untouched."""
    shard, stripe, off = xrs_amd.batch_layout(size, d + p)
    assert (shard, stripe) == xrs_amd.batch_strides(size, d + p)
    assert off == (16 - (size // 2) % 16) % 16
    buf = rng.integers(0, 256, size=off + n * stripe, dtype=np.uint8)
    x, o = xrs_amd.XRS(d, p), OracleXRS(d, p)

    def rows(b, s):
        return [b[off + s * stripe + i * shard:][:size] for i in range(d + p)]

    ref = buf.copy()
    for s in range(n):
        v = [r.copy() for r in rows(ref, s)]
        o.encode(v)
        for i in range(d + p):
            ref[off + s * stripe + i * shard:][:size] = v[i]
    t = to_dev(buf, cuda)
    base = t.data_ptr() + off
    x.encode_batched(base, size, shard, stripe, n, stream())
    torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy(), ref)  # gaps included
    for k in range(d):
        t = to_dev(ref, cuda)
        tv = t[off:off + n * stripe].view(n, stripe)
        tv[:, k * shard:k * shard + size] = 0x5A
        x.reconst_one_batched(t.data_ptr() + off, size, shard, stripe, n, k, stream())
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy(), ref), k
    lost = [0, d - 1]
    has = [i for i in range(d + p) if i not in lost]
    exp = ref.copy()
    for s in range(n):
        v = [r.copy() for r in rows(exp, s)]
        for i in lost:
            v[i][:] = 0
        o.reconst(v, has, lost)
        for i in range(d + p):
            exp[off + s * stripe + i * shard:][:size] = v[i]
    t = to_dev(ref, cuda)
    tv = t[off:off + n * stripe].view(n, stripe)
    for i in lost:
        tv[:, i * shard:i * shard + size] = 0
    x.reconst_batched(t.data_ptr() + off, size, shard, stripe, n, has, lost, stream())
    torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy(), exp)
