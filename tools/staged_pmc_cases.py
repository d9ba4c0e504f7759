#!/usr/bin/env python3
"""Staged general-Reconst launches for rocprofv3 --pmc passes (HBM bytes per
launch vs the bytes the launch must move): 12+4 with 2 / 3 / 4 lost data
vects (wave-specialised kernel for 2-3, one-wave compile-time kernel for 4)
and a lost data + parity pattern, at 4 KiB and 1 MiB vects, and 16+4 with 2
lost data vects (wide b-side kernel).  Each case: 3 launches on a 4 GiB batch,
preceded by one Encode.  Prints one JSON line per case with the expected
bytes moved per launch (reads + writes, side effects included), which
tools/pmc_by_kernel.py output is compared against.

    rocprofv3 --pmc FETCH_SIZE -d OUT -o pmc --output-format csv -- python tools/staged_pmc_cases.py
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xrs_amd  # noqa: E402


def moved_halves(d, p, lost, need):
    """Half-rows a clean staged pass reads and writes (xrs.go:236-320)."""
    xs = {}
    for c in range(d):  # makeXORSet: data c rides on parity d + 1 + c mod (p - 1)
        xs.setdefault(d + 1 + c % (p - 1), []).append(c)
    has = [i for i in range(d + p) if i not in lost]
    first = has[:d]
    a_rows = set(first)
    b_rows = set(first)
    writes = len(lost)  # lost a-halves
    for h in range(d + 1, d + p):
        if h in has and xs.get(h):
            b_rows.add(h)
            writes += 1  # retrieveRS write-back
            a_rows |= {j for j in xs[h] if j in has}
    for u in need:
        if u > d and xs.get(u):
            a_rows |= {j for j in xs[u] if j in has}
    writes += len(need)
    return len(a_rows) + len(b_rows), writes


def main():
    s = torch.cuda.current_stream().cuda_stream
    cases = [(12, 4, 4096, [0, 1]), (12, 4, 4096, [0, 1, 2]), (12, 4, 4096, [0, 1, 2, 3]),
             (12, 4, 4096, [0, 13]), (12, 4, 1 << 20, [0, 1]), (12, 4, 1 << 20, [0, 1, 2]),
             (12, 4, 1 << 20, [0, 1, 2, 3]), (16, 4, 4096, [0, 1])]
    for d, p, size, lost in cases:
        x = xrs_amd.XRS(d, p)
        n = (4 << 30) // ((d + p) * size)
        buf = torch.randint(0, 256, (n * (d + p) * size,), dtype=torch.uint8, device="cuda")
        x.encode_batched(buf.data_ptr(), size, size, (d + p) * size, n, s)
        has = [i for i in range(d + p) if i not in lost]
        for _ in range(3):
            x.reconst_batched(buf.data_ptr(), size, size, (d + p) * size, n, has, lost, s)
        torch.cuda.synchronize()
        r, w = moved_halves(d, p, lost, lost)
        print(json.dumps({"codec": f"{d}+{p}", "vect_bytes": size, "lost": lost, "stripes": n,
                          "read_halves": r, "write_halves": w,
                          "moved_bytes_per_launch": (r + w) * (size // 2) * n}), flush=True)
        del buf


if __name__ == "__main__":
    main()
