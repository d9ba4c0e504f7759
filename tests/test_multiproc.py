"""World-size-2 gloo tests (CPU) of the multi-GPU path: the stripe split and
the barrier/max-time bracket bench.py uses.  The per-rank compute is the CPU
oracle here (the GPU box runs the kernels; 8-GPU runs are the driver's)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from xrs_amd.dist import stripe_range


def test_stripe_range_partitions():
    for n in (0, 1, 7, 8, 65536, 65537):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                s, c = stripe_range(n, r, world)
                seen.extend(range(s, s + c))
            assert seen == list(range(n))
    with pytest.raises(ValueError):
        stripe_range(8, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_stripes, size, out_dir):
    import torch
    import torch.distributed as dist

    from oracle.oracle_c import OracleXRS
    from xrs_amd.dist import stripe_range, timed_steps

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.Generator(np.random.PCG64(42))
    full = rng.integers(0, 256, size=(n_stripes, 16, size), dtype=np.uint8)
    start, count = stripe_range(n_stripes, rank, world)
    mine = full[start:start + count].copy()
    o = OracleXRS(12, 4)

    def step(i):
        o.encode_batch(mine, size, count)

    own, mx = timed_steps(step, steps=3, warmup=1, sync=lambda: None, device="cpu")
    assert mx >= own
    t = torch.from_numpy(mine.reshape(-1).copy())
    sizes = [stripe_range(n_stripes, r, world)[1] * 16 * size for r in range(world)]
    gathered = [torch.empty(s_, dtype=torch.uint8) for s_ in sizes]
    # only the test gathers results; the benchmark path has no data collective
    dist.all_gather(gathered, t) if len(set(sizes)) == 1 else [
        dist.broadcast(gathered[r].copy_(t) if r == rank else gathered[r], src=r)
        for r in range(world)]
    if rank == 0:
        got = np.concatenate([g.numpy() for g in gathered]).reshape(n_stripes, 16, size)
        ref = full.copy()
        o.encode_batch(ref, size, n_stripes)
        np.save(os.path.join(out_dir, "ok.npy"), np.array([np.array_equal(got, ref), mx]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_stripes", [64, 65])
def test_two_rank_split_encode_gloo(tmp_path, n_stripes):
    mp.spawn(_worker, args=(2, _free_port(), n_stripes, 4096, str(tmp_path)), nprocs=2, join=True)
    ok, mx = np.load(tmp_path / "ok.npy")
    assert ok == 1 and mx > 0
