"""GPU tests of the XCD-aware block order (kernels.hip logical_block): every
order (plain, several K, one range per XCD) must process every block exactly
once, for grids that are and are not multiples of 8*K, against the oracle."""
import numpy as np
import pytest

import xrs_amd
from oracle.oracle_c import OracleXRS

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

D, P = 12, 4
# (vect size, stripes): blocks per launch = stripes * size / 2 / 16 / 256
SHAPES = [
    (4096, 1),       # half a block
    (4096, 15),      # 7.5 blocks: fewer than 8
    (4096, 513),     # 256.5 blocks: partial group and partial block
    (65536, 37),     # 296 blocks
    (1 << 20, 9),    # 2304 blocks (half >= 256 KiB: rows use K = 128)
]
ORDERS = ["0", "1", "3", "32", "128", "full", "100000"]


def batch(rng, size, n):
    host = rng.integers(0, 256, size=(n, D + P, size), dtype=np.uint8)
    return host, torch.from_numpy(host).cuda()


@pytest.mark.parametrize("order", ORDERS)
@pytest.mark.parametrize("size,n", SHAPES)
def test_encode_and_reconst_one_every_order(rng, monkeypatch, order, size, n):
    monkeypatch.setenv("XRS_BLOCK_ORDER", order)
    host, t = batch(rng, size, n)
    s = torch.cuda.current_stream().cuda_stream
    x = xrs_amd.XRS(D, P)
    x.encode_batched(t.data_ptr(), size, size, (D + P) * size, n, s)
    ref = host.copy()
    OracleXRS(D, P).encode_batch(ref, size, n)
    torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy(), ref)
    k = 7
    t[:, k].fill_(0xA5)
    x.reconst_one_batched(t.data_ptr(), size, size, (D + P) * size, n, k, s)
    torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy(), ref)


@pytest.mark.parametrize("variant", ["late", "late_one_wave", "0"])
@pytest.mark.parametrize("order", ["0", "32", "full"])
@pytest.mark.parametrize("size,n", [(4096, 513), (1 << 20, 9)])
def test_staged_reconst_every_order(rng, monkeypatch, variant, order, size, n):
    """Three lost data vects through every staged kernel variant (late: the
    wave-specialised kernel; late_one_wave: the compile-time one-wave kernel;
    0: all loads first), side effects included."""
    monkeypatch.setenv("XRS_BLOCK_ORDER", order)
    monkeypatch.setenv("XRS_STAGED_LATE", "0" if variant == "0" else "1")
    monkeypatch.setenv("XRS_STAGED_WS", "0" if variant == "late_one_wave" else "")
    host, t = batch(rng, size, n)
    o = OracleXRS(D, P)
    o.encode_batch(host, size, n)
    t.copy_(torch.from_numpy(host))
    need = [0, 4, 9]
    has = [i for i in range(D + P) if i not in need]
    x = xrs_amd.XRS(D, P)
    s = torch.cuda.current_stream().cuda_stream
    x.reconst_batched(t.data_ptr(), size, size, (D + P) * size, n, has, need, s)
    torch.cuda.synchronize()
    got = t.cpu().numpy()
    for st in range(n):
        v = [host[st, i].copy() for i in range(D + P)]
        o.reconst(v, has, need)
        for i in range(D + P):
            assert np.array_equal(got[st, i], v[i]), (st, i)
