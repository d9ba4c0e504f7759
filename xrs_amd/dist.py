"""Multi-GPU plumbing for the codec: stripes are independent, so a batch is a
plain contiguous split across ranks (one process per GPU) and no collective
touches the data path.  The only cross-rank operations are the barrier and
the max-time reduction that bracket a timed region (bench.py).

Works with any torch.distributed backend: "nccl" (RCCL over xGMI) on the GPU
box, "gloo" in the CPU tests.
"""
from __future__ import annotations

import time
from typing import Callable, Tuple


def stripe_range(n_stripes: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous balanced split: (first stripe, count) owned by `rank`."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(n_stripes, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def timed_steps(step: Callable[[int], None], steps: int, warmup: int,
                sync: Callable[[], None], device=None) -> Tuple[float, float]:
    """Run `warmup` untimed steps, then time exactly `steps` steps bracketed by
    barrier + sync on both sides.  Returns (own elapsed, max over ranks) in s."""
    import torch
    import torch.distributed as dist

    ddp = dist.is_available() and dist.is_initialized()
    for i in range(warmup):
        step(i)
    sync()
    if ddp:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    sync()
    elapsed = time.perf_counter() - t0
    if ddp:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return elapsed, float(t.item())
    return elapsed, elapsed
