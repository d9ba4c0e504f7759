"""One rank of tests/test_multiproc.py: the same xrs_amd.dist calls bench.py
makes (resolve_world, init, stripe_range, timed_steps), over gloo on CPU, with
the CPU oracle as the per-rank compute (the GPU box runs the kernels).

usage: python tests/_rank_worker.py OUT_DIR N_STRIPES SIZE [FAIL_RANK]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    out_dir, n_stripes, size = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    fail_rank = int(sys.argv[4]) if len(sys.argv) > 4 else -1
    import torch
    import torch.distributed as dist

    from oracle.oracle_c import OracleXRS
    from xrs_amd import dist as xdist

    w = xdist.resolve_world(None)
    if w.rank == fail_rank:
        sys.exit(3)
    xdist.init(w, "gloo")
    rng = np.random.Generator(np.random.PCG64(42))
    full = rng.integers(0, 256, size=(n_stripes, 16, size), dtype=np.uint8)
    start, count = xdist.stripe_range(n_stripes, w.rank, w.world)
    mine = full[start:start + count].copy()
    o = OracleXRS(12, 4)
    calls = []

    def step(i):
        calls.append(i)
        o.encode_batch(mine, size, count)

    secs = xdist.timed_steps(step, steps=3, warmup=1, sync=lambda: None)
    assert calls == [0, 0, 1, 2], calls  # 1 warmup + exactly 3 timed steps
    one = xdist.timed_region(lambda: o.encode_batch(mine, size, count), sync=lambda: None)
    # only the test gathers results; the benchmark path has no data collective
    t = torch.from_numpy(mine.reshape(-1).copy())
    sizes = [xdist.stripe_range(n_stripes, r, w.world)[1] * 16 * size for r in range(w.world)]
    gathered = [torch.empty(s_, dtype=torch.uint8) for s_ in sizes]
    for r in range(w.world):
        buf = gathered[r]
        if r == w.rank:
            buf.copy_(t)
        dist.broadcast(buf, src=r)
    if w.rank == 0:
        got = np.concatenate([g.numpy() for g in gathered]).reshape(n_stripes, 16, size)
        ref = full.copy()
        o.encode_batch(ref, size, n_stripes)
        with open(os.path.join(out_dir, "result.json"), "w") as f:
            json.dump({"ok": bool(np.array_equal(got, ref)), "rank_seconds": secs,
                       "region_seconds": one, "world": w.world,
                       "counts": [xdist.stripe_range(n_stripes, r, w.world)[1]
                                  for r in range(w.world)]}, f)
    xdist.barrier()
    xdist.finalize()


if __name__ == "__main__":
    main()
