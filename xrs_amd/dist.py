"""Multi-GPU harness of the codec: one process per GPU, stripes split by plain
contiguous ranges, no collective on the data path.

Stripes are independent (xrs.go has no cross-stripe state: every method works
on one stripe's `vects`), so a batch partitions across ranks with no exchange
step.  The only cross-rank operations are the barrier and the per-rank time
gather that bracket a timed region.  bench.py runs everything it times through
this module, and tests/test_multiproc.py runs the same functions over gloo on
CPU, so what the 8-GPU run executes is what the CPU tests cover:

  * `resolve_world(gpus)`  -- rank / world / local rank from the torchrun env,
    checked against `--gpus`;
  * `launch_local(n, argv)` -- `bench.py --gpus N` without torchrun: the parent
    starts N rank processes (before it touches the GPU) and waits for them;
  * `stripe_range`          -- the contiguous split;
  * `timed_steps` / `timed_region` -- warmup, barrier + sync on both sides of
    exactly K steps, every rank's elapsed time gathered (max = the job time).

Works with any torch.distributed backend.  bench.py uses "gloo" by default:
the bracket is a host barrier and a gather of a few floats, no shard byte
crosses ranks, so an RCCL communicator would carry nothing ("nccl" still
works, XRS_DIST_BACKEND=nccl).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple


@dataclass(frozen=True)
class World:
    rank: int
    world: int
    local: int
    launched: bool  # True: WORLD_SIZE came from a launcher (torchrun or launch_local)


class WorldMismatch(ValueError):
    """--gpus disagrees with the launcher's WORLD_SIZE."""


def resolve_world(gpus: Optional[int], env=None) -> World:
    """Rank layout of this process.  With WORLD_SIZE set (torchrun, or a child
    of launch_local) it must equal `gpus` when `gpus` is given; without it the
    process is rank 0 of a world of `gpus` (the caller spawns the others)."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if gpus is not None and gpus != world:
            raise WorldMismatch(
                f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks; "
                f"they must agree (one rank per GPU)")
        return World(int(env.get("RANK", 0)), world, int(env.get("LOCAL_RANK", env.get("RANK", 0))),
                     True)
    world = 1 if gpus is None else int(gpus)
    if world < 1:
        raise WorldMismatch(f"--gpus must be >= 1, got {world}")
    return World(0, world, 0, False)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_local(n: int, argv: Sequence[str], env=None, timeout: Optional[float] = None) -> int:
    """Start `n` rank processes of `argv` on this node (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in their env) and wait.
    The caller must not have touched the GPU.  Returns the first non-zero exit
    code (after stopping the remaining ranks), else 0."""
    base = dict(os.environ if env is None else env)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n))
    procs: List[subprocess.Popen] = []

    def stop(live):  # exactly the processes this call started
        for p in live:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in live:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    # A SIGTERM to this parent (a driver's time limit) must not orphan ranks
    # that hold GPUs: turn it into an exception, so the finally below stops them.
    def on_term(signum, frame):
        raise SystemExit(128 + signum)

    old = signal.signal(signal.SIGTERM, on_term)
    rc = 0
    live: List[subprocess.Popen] = []
    try:
        for r in range(n):
            e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
            procs.append(subprocess.Popen(list(argv), env=e))
        t0 = time.monotonic()
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
            if rc != 0 or (timeout is not None and time.monotonic() - t0 > timeout):
                if rc == 0:
                    rc = 124
                break
            time.sleep(0.05)
    finally:
        stop([p for p in procs if p.poll() is None])
        signal.signal(signal.SIGTERM, old)
    return rc


class _StdoutToStderr:
    """fd 1 -> fd 2 for the duration: gloo's C++ side prints "[Gloo] Rank r
    is connected to ..." on stdout while the group connects, and rank 0's
    stdout must carry only the bench's JSON line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def init(w: World, backend: str, device=None) -> None:
    """Join the process group (world > 1 only); the first barrier connects
    every pair, so it runs inside the stdout redirect too."""
    if w.world <= 1:
        return
    import torch.distributed as dist

    with _StdoutToStderr():
        if backend == "nccl":
            dist.init_process_group("nccl", rank=w.rank, world_size=w.world, device_id=device)
        else:
            dist.init_process_group(backend, rank=w.rank, world_size=w.world)
        dist.barrier()


def finalize() -> None:
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def _ddp() -> bool:
    import torch.distributed as dist

    return dist.is_available() and dist.is_initialized()


def barrier() -> None:
    if _ddp():
        import torch.distributed as dist

        dist.barrier()


def stripe_range(n_stripes: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous balanced split: (first stripe, count) owned by `rank`."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(n_stripes, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def gather_seconds(elapsed: float, device=None) -> List[float]:
    """Every rank's `elapsed`, indexed by rank (one slot each, summed)."""
    if not _ddp():
        return [float(elapsed)]
    import torch
    import torch.distributed as dist

    t = torch.zeros(dist.get_world_size(), dtype=torch.float64,
                    device=device if device is not None else "cpu")
    t[dist.get_rank()] = elapsed
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.cpu()]


class SharedDevice(RuntimeError):
    """Two ranks resolved to the same GPU outside a labelled rehearsal."""


def rehearsal_env(env=None) -> bool:
    """XRS_REHEARSAL=1: ranks may share a card (one-GPU rehearsals of the
    multi-rank path); the bench line then says "shared_gpu": true."""
    env = os.environ if env is None else env
    return env.get("XRS_REHEARSAL", "") not in ("", "0")


def gather_objects(obj) -> list:
    """Every rank's picklable `obj`, indexed by rank (over the process group;
    [obj] without one)."""
    if not _ddp():
        return [obj]
    import torch.distributed as dist

    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def check_distinct_devices(rank_devices: Sequence[dict], rehearsal: bool) -> bool:
    """True when two ranks share a GPU (same "pci" address).  Outside a
    rehearsal that is an error: a line claiming N GPUs must have run on N."""
    seen = {}
    shared = False
    for d in rank_devices:
        key = d["pci"]
        if key in seen:
            shared = True
            if not rehearsal:
                raise SharedDevice(
                    f"ranks {seen[key]} and {d['rank']} run on the same GPU ({key}); one rank "
                    f"per GPU is required (XRS_REHEARSAL=1 for a labelled one-card rehearsal)")
        else:
            seen[key] = d["rank"]
    return shared


def timed_steps(step: Callable[[int], None], steps: int, warmup: int, sync: Callable[[], None],
                device=None) -> List[float]:
    """`warmup` untimed steps, then exactly `steps` steps bracketed by barrier +
    sync on both sides.  Returns every rank's elapsed seconds (max = job time)."""
    for i in range(warmup):
        step(i)
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    sync()
    elapsed = time.perf_counter() - t0
    barrier()
    return gather_seconds(elapsed, device)


def timed_region(fn: Callable[[], None], sync: Callable[[], None], device=None) -> List[float]:
    """One call of `fn` bracketed like a step; every rank's elapsed seconds."""
    return timed_steps(lambda i: fn(), 1, 0, sync, device)

