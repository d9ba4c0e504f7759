"""Randomised parity of the batched device API against the oracle.

Each case draws a codec (d, p), a vect size (even, 2 B to 40 KiB), a stripe
count, a layout (shard and stripe strides with random padding, and a base
offset 0..15 so both the 16-byte and the byte-granular kernels run) and one
operation (Encode, ReconstOne, Reconst with random losses and needs, Update,
Replace).  The GPU buffer after the call must equal the oracle applied stripe
by stripe to a host copy, byte for byte, including every byte outside the
shards (nothing else may be written).  Seeded; bounded to a few seconds.
XRS_FUZZ_SEEDS=N runs N seeds per test instead of 10 (long campaigns);
XRS_FUZZ_BASE=B starts the seeds at B (fresh cases for a new campaign);
XRS_FUZZ_BIG=1 adds 128 KiB-1 MiB vects, XRS_FUZZ_GRID=1 full grids."""
import os

import numpy as np
import pytest

import xrs_amd
from oracle.oracle_c import OracleXRS

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

CODECS = [(12, 4), (10, 4), (6, 3), (4, 2), (5, 5), (20, 4), (1, 2), (30, 6), (3, 9), (16, 8)]
OPS = ["encode", "reconst_one", "reconst", "update", "replace"]
SEEDS = int(os.environ.get("XRS_FUZZ_SEEDS", "10"))
BASE = int(os.environ.get("XRS_FUZZ_BASE", "0"))


BIG = os.environ.get("XRS_FUZZ_BIG") == "1"  # long campaigns: also 128 KiB-1 MiB vects
# every other case on a grid of >= 256 blocks, where the bandwidth kernels
# (wave-specialised staged Reconst, late / XCD-ordered launches) run
GRID = os.environ.get("XRS_FUZZ_GRID") == "1"


def draw_case(rng):
    d, p = CODECS[int(rng.integers(0, len(CODECS)))]
    size = int(rng.choice([2, 34, 1024, 1026, 4096, 4112, 6000, 40960]))
    n = int(rng.integers(1, 40))
    if BIG and rng.integers(0, 4) == 0:
        size = int(rng.choice([131072, 131074, 262160, 1048576, 1048578]))
        n = int(rng.integers(1, 4))
    if GRID and rng.integers(0, 2) == 0:
        size = int(rng.choice([4096, 4112, 8192, 40960, 65536]))
        n = -(-65536 * 32 // size) + int(rng.integers(0, 64))  # >= 65,536 16-byte lanes
    shard = size + int(rng.choice([0, 0, 2, 16, 256]))
    stripe = (d + p) * shard + int(rng.choice([0, 0, 6, 64]))
    base = int(rng.choice([0, 0, 0, 1, 8, 14, 15]))  # 14, 15: xrs_batch_layout offsets
    return d, p, size, n, shard, stripe, base, OPS[int(rng.integers(0, len(OPS)))]


def vects_of(buf, base, s, shard, stripe, size, count, first=0):
    o = base + s * stripe
    return [buf[o + (first + i) * shard: o + (first + i) * shard + size] for i in range(count)]


@pytest.mark.parametrize("seed", range(SEEDS))
def test_batched_fuzz_vs_oracle(seed):
    rng = np.random.Generator(np.random.PCG64(9000 + BASE + seed))
    dev = torch.device("cuda:0")
    s_ = torch.cuda.current_stream().cuda_stream
    for case in range(30):
        d, p, size, n, shard, stripe, base, op = draw_case(rng)
        x, o = xrs_amd.XRS(d, p), OracleXRS(d, p)
        total = base + n * stripe + 64
        host = rng.integers(0, 256, size=total, dtype=np.uint8)
        # start from encoded stripes (reconstruction needs consistent parity)
        for s in range(n):
            o.encode(vects_of(host, base, s, shard, stripe, size, d + p))
        ref = host.copy()
        t = torch.from_numpy(host).to(dev)
        ptr = t.data_ptr() + base
        tag = (seed, case, d, p, size, n, shard, stripe, base, op)
        if op == "encode":
            for s in range(n):  # garbage parity in, must be overwritten
                for v in vects_of(host, base, s, shard, stripe, size, p, first=d):
                    v[:] = rng.integers(0, 256, size=size, dtype=np.uint8)
            t.copy_(torch.from_numpy(host))
            x.encode_batched(ptr, size, shard, stripe, n, s_)
        elif op == "reconst_one":
            k = int(rng.integers(0, d))
            for s in range(n):
                vects_of(host, base, s, shard, stripe, size, 1, first=k)[0][:] = 0x5A
            t.copy_(torch.from_numpy(host))
            x.reconst_one_batched(ptr, size, shard, stripe, n, k, s_)
        elif op == "reconst":
            lost = [int(v) for v in rng.permutation(d + p)[: int(rng.integers(0, p + 1))]]
            need = lost[: int(rng.integers(0, len(lost) + 1))]
            has = [i for i in range(d + p) if i not in lost]
            for s in range(n):
                for i in lost:
                    vects_of(host, base, s, shard, stripe, size, 1, first=i)[0][:] = 0xA5
            ref = host.copy()
            t.copy_(torch.from_numpy(host))
            x.reconst_batched(ptr, size, shard, stripe, n, has, need, s_)
            for s in range(n):
                o.reconst(vects_of(ref, base, s, shard, stripe, size, d + p), has, need)
        elif op == "update":
            row = int(rng.integers(0, d))
            new = rng.integers(0, 256, size=n * size, dtype=np.uint8)
            tn = torch.from_numpy(new).to(dev)
            old_ptr = ptr + row * shard
            x.update_batched(old_ptr, stripe, tn.data_ptr(), size, size, row, ptr + d * shard,
                             shard, stripe, n, s_)
            for s in range(n):
                old = vects_of(ref, base, s, shard, stripe, size, 1, first=row)[0]
                o.update(old, new[s * size:(s + 1) * size],
                         row, vects_of(ref, base, s, shard, stripe, size, p, first=d))
        else:  # replace
            k = int(rng.integers(1, d + 1))
            rows = [int(v) for v in rng.permutation(d)[:k]]
            x.replace_batched(ptr, shard, stripe, rows, size, ptr + d * shard, shard, stripe, n,
                              s_)
            for s in range(n):  # data[i] (for row rows[i]) is vect i of the stripe
                o.replace(vects_of(ref, base, s, shard, stripe, size, k), rows,
                          vects_of(ref, base, s, shard, stripe, size, p, first=d))
        torch.cuda.synchronize()
        got = t.cpu().numpy()
        if not np.array_equal(got, ref):
            bad = np.nonzero(got != ref)[0]
            raise AssertionError(f"{tag}: {len(bad)} bytes differ, first at {bad[0]}")


@pytest.mark.parametrize("seed", range(max(1, SEEDS * 2 // 5)))
def test_sync_fuzz_vs_oracle(seed):
    """The per-stripe sync API (host vects: separate, oddly aligned numpy
    slices, sizes spanning the zero-copy / pinned / direct staging modes) on
    random codecs and operations, against the oracle."""
    rng = np.random.Generator(np.random.PCG64(9500 + BASE + seed))
    for case in range(30):
        d, p = CODECS[int(rng.integers(0, len(CODECS)))]
        size = int(rng.choice([2, 34, 4096, 4112, 65538, 300000, 600002]))
        x, o = xrs_amd.XRS(d, p), OracleXRS(d, p)

        def fresh(count):  # separate buffers at odd offsets
            out = []
            for _ in range(count):
                off = int(rng.integers(0, 16))
                out.append(rng.integers(0, 256, size=size + off, dtype=np.uint8)[off:])
            return out

        v = fresh(d + p)
        o.encode(v)
        op = OPS[int(rng.integers(0, len(OPS)))]
        a, b = [t.copy() for t in v], [t.copy() for t in v]
        tag = (seed, case, d, p, size, op)
        if op == "encode":
            for t in a[d:]:
                t[:] = 0x33
            x.encode(a)
        elif op == "reconst_one":
            k = int(rng.integers(0, d))
            a[k][:] = 0
            x.reconst_one(a, k)
        elif op == "reconst":
            lost = [int(t) for t in rng.permutation(d + p)[: int(rng.integers(0, p + 1))]]
            need = lost[: int(rng.integers(0, len(lost) + 1))]
            has = [i for i in range(d + p) if i not in lost]
            for i in lost:
                a[i][:] = 0xA5
                b[i][:] = 0xA5
            x.reconst(a, has, need)
            o.reconst(b, has, need)
        elif op == "update":
            row = int(rng.integers(0, d))
            new = fresh(1)[0]
            x.update(a[row], new, row, a[d:])
            o.update(b[row], new, row, b[d:])
        else:
            k = int(rng.integers(1, d + 1))
            rows = [int(t) for t in rng.permutation(d)[:k]]
            data = fresh(k)
            x.replace(data, rows, a[d:])
            o.replace(data, rows, b[d:])
        assert all(np.array_equal(s, t) for s, t in zip(a, b)), tag


@pytest.mark.parametrize("d,p,size", [(12, 4, 4096), (12, 4, 1026), (12, 4, 34), (30, 6, 4096),
                                      (1, 2, 4096), (10, 4, 1 << 20), (3, 9, 2)])
def test_update_rows_batched_vs_oracle(d, p, size):
    """xrs_update_rows_batched: every stripe its own data row (rows beyond one
    launch's 24-row chunk and parity beyond one 4-output group included);
    stripes whose row is not a data row (-1, d) are left untouched."""
    rng = np.random.Generator(np.random.PCG64(7000 + d * 31 + p + size))
    dev = torch.device("cuda:0")
    s_ = torch.cuda.current_stream().cuda_stream
    x, o = xrs_amd.XRS(d, p), OracleXRS(d, p)
    n = 200 if size < (1 << 20) else 6
    stripe = (d + p) * size
    host = rng.integers(0, 256, size=n * stripe, dtype=np.uint8)
    for s in range(n):
        o.encode(vects_of(host, 0, s, size, stripe, size, d + p))
    new = rng.integers(0, 256, size=n * size, dtype=np.uint8)
    rows = rng.integers(0, d, size=n).astype(np.int32)
    rows[::17] = -1
    rows[5::23] = d
    ref = host.copy()
    for s in range(n):
        if 0 <= rows[s] < d:
            o.update(vects_of(ref, 0, s, size, stripe, size, 1, first=int(rows[s]))[0],
                     new[s * size:(s + 1) * size], int(rows[s]),
                     vects_of(ref, 0, s, size, stripe, size, p, first=d))
    # old data row of stripe s: its own row (a clamped row for skipped stripes)
    olds = np.stack([vects_of(host, 0, s, size, stripe, size, 1,
                              first=int(min(max(rows[s], 0), d - 1)))[0] for s in range(n)])
    t = torch.from_numpy(host).to(dev)
    to = torch.from_numpy(olds.reshape(-1)).to(dev)
    tn = torch.from_numpy(new).to(dev)
    tr = torch.from_numpy(rows).to(dev)
    x.update_rows_batched(to.data_ptr(), size, tn.data_ptr(), size, size, tr.data_ptr(),
                          t.data_ptr() + d * size, size, stripe, n, s_)
    torch.cuda.synchronize()
    got = t.cpu().numpy()
    assert np.array_equal(got, ref), np.nonzero(got != ref)[0][:5]
