#!/usr/bin/env python3
"""Staged multi-loss Reconst at large halves: why do 8 MiB
vects stream slower than 2 MiB ones, and 3 / 4 lost slower than 2 at 1 MiB?

Each case is one 12+4 launch shape on a ~4 GiB batch laid out by
xrs_batch_layout, with the kernel choice forced by environment knobs read at
launch time (XRS_WSP=0: the one-shot wave-specialised kernel, =512: the
persistent one).  Per case: 2 warm-up launches, then ROUNDS timed launches
(HIP events on the launch stream), one JSON line with the median rate of the
bytes the launch moves (reads + writes, side effects included: 16.5 / 17 /
17.5 vect-sizes per stripe for 2 / 3 / 4 lost data vects).  Run it bare for
rates, or under rocprofv3 --pmc for counters per kernel (tools/pmc_generic.py).

    python tools/staged_big_cases.py [CASES=A,B,...] [ROUNDS=7]
"""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xrs_amd  # noqa: E402

D, P = 12, 4
MIB = 1 << 20
# name: (op, vect bytes, lost data vects, env)
CASES = {
    "A": ("reconst", 2 * MIB, 2, {"XRS_WSP": "0"}),
    "B": ("reconst", 2 * MIB, 2, {"XRS_WSP": "512"}),
    "C": ("reconst", 8 * MIB, 2, {"XRS_WSP": "0"}),
    "D": ("reconst", 8 * MIB, 2, {"XRS_WSP": "512"}),
    "E": ("reconst", 1 * MIB, 3, {}),
    "F": ("reconst", 1 * MIB, 4, {}),
    "G": ("reconst", 1 * MIB, 2, {}),
    "H": ("encode", 8 * MIB, 0, {}),
    "I": ("reconst_one", 8 * MIB, 1, {}),
    "J": ("reconst", 8 * MIB, 3, {}),
}
MOVED = {0: 16.0, 1: 9.0, 2: 16.5, 3: 17.0, 4: 17.5}  # vect-sizes moved per stripe


def main():
    names = os.environ.get("CASES", ",".join(CASES)).split(",")
    rounds = int(os.environ.get("ROUNDS", "7"))
    x = xrs_amd.XRS(D, P)
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    for name in names:
        op, size, lost, env = CASES[name]
        shard, stripe, bo = xrs_amd.batch_layout(size, D + P)
        n = max(1, (4 << 30) // stripe)
        buf = torch.randint(0, 256, (n * stripe + bo + 16,), dtype=torch.uint8, device="cuda")
        b = buf.data_ptr() + bo
        x.encode_batched(b, size, shard, stripe, n, s)
        for k, v in env.items():
            os.environ[k] = v
        has = list(range(lost, D + P))
        need = list(range(lost))
        if op == "encode":
            fn = lambda: x.encode_batched(b, size, shard, stripe, n, s)  # noqa: E731
        elif op == "reconst_one":
            fn = lambda: x.reconst_one_batched(b, size, shard, stripe, n, 0, s)  # noqa: E731
        else:
            fn = lambda: x.reconst_batched(b, size, shard, stripe, n, has, need, s)  # noqa: E731
        xrs_amd.trace_kernels(True)
        for _ in range(2):
            fn()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ms = []
        for _ in range(rounds):
            ev[0].record(stream)
            fn()
            ev[1].record(stream)
            ev[1].synchronize()
            ms.append(ev[0].elapsed_time(ev[1]))
        xrs_amd.trace_kernels(False)
        for k in env:
            os.environ.pop(k, None)
        med = statistics.median(ms)
        moved = MOVED[lost] * size * n
        print(json.dumps({"case": name, "op": op, "vect_bytes": size, "lost": lost, "env": env,
                          "stripes": n, "ms": round(med, 4),
                          "moved_gbs": round(moved / med / 1e6, 1),
                          "frac_moved": round(moved / med / 1e6 / 8000.0, 4),
                          "kernels": list(xrs_amd.traced_kernels())}), flush=True)
        del buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
