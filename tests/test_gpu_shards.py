"""GPU tests of the per-shard pointer-table API (xrs_*_shards): each shard in
its own allocation (one buffer per disk, shard-major), and - when two GPUs
are visible - shards on a peer GPU read over xGMI (cross-GPU repair)."""
import numpy as np
import pytest

import xrs_amd
from oracle.oracle_c import OracleXRS

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
D, P = 12, 4


def shard_major(rng, n, size):
    return rng.integers(0, 256, size=(D + P, n, size), dtype=np.uint8)


@pytest.mark.parametrize("size,n", [(4096, 300), (1 << 20, 6), (1030, 77)])
def test_shards_encode_reconst(rng, size, n):
    host = shard_major(rng, n, size)
    dev = [torch.from_numpy(host[i].copy()).cuda() for i in range(D + P)]  # separate allocations
    ptrs = [t.data_ptr() for t in dev]
    x = xrs_amd.XRS(D, P)
    s = torch.cuda.current_stream().cuda_stream
    x.encode_shards(ptrs, size, size, n, s)
    torch.cuda.synchronize()
    o = OracleXRS(D, P)
    ref = np.ascontiguousarray(host.transpose(1, 0, 2))  # [n][16][size]
    o.encode_batch(ref, size, n)
    got = np.stack([t.cpu().numpy() for t in dev]).transpose(1, 0, 2)
    assert np.array_equal(got, ref)
    # ReconstOne with every shard outside the need set passed as NULL
    for k in (0, 5, 11):
        a_need, b_need = x.get_need_vects(k)
        dev[k].zero_()
        table = [ptrs[i] if (i < D or i in b_need or i == k or i in a_need) else None
                 for i in range(D + P)]
        x.reconst_one_shards(table, size, size, n, k, s)
        torch.cuda.synchronize()
        assert np.array_equal(dev[k].cpu().numpy(), ref[:, k]), k
    # general Reconst: lose 2 data + 1 parity
    lost = [2, 9, 14]
    for t in lost:
        dev[t].fill_(0x33)
    has = [i for i in range(D + P) if i not in lost]
    x.reconst_shards(ptrs, size, size, n, has, lost, s)
    torch.cuda.synchronize()
    for t in lost:
        assert np.array_equal(dev[t].cpu().numpy(), ref[:, t]), t


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                    reason="cross-GPU repair needs two GPUs")
def test_cross_gpu_reconst_one(rng):
    """Shards spread over GPU 0 and 1; ReconstOne runs on GPU 0 and reads the
    GPU-1 shards over xGMI peer access."""
    size, n = 1 << 20, 8
    host = shard_major(rng, n, size)
    ref = np.ascontiguousarray(host.transpose(1, 0, 2))
    OracleXRS(D, P).encode_batch(ref, size, n)
    enc = np.ascontiguousarray(ref.transpose(1, 0, 2))
    assert xrs_amd.lib().xrs_enable_peer_access(0, 1) == 0
    dev = [torch.from_numpy(enc[i].copy()).to(f"cuda:{i % 2}") for i in range(D + P)]
    torch.cuda.set_device(0)
    x = xrs_amd.XRS(D, P)
    k = 4
    dev[k].zero_()
    x.reconst_one_shards([t.data_ptr() for t in dev], size, size, n, k,
                         torch.cuda.current_stream(0).cuda_stream)
    torch.cuda.synchronize(0)
    assert np.array_equal(dev[k].cpu().numpy(), enc[k])
