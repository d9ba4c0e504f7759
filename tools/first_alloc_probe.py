#!/usr/bin/env python3
"""Is 12+4 Encode @ 4 KiB slower on the first buffer a process allocates?
(tools/refbench.py, which times it first thing, read 0.66-0.69 of 8 TB/s on
two boxes; bench.py and tools/b2b_probe.py read 0.74-0.75.)  Times Encode on
buffer A right after allocation, then after a warm period, then A and a
second buffer B interleaved; median ms of 10-launch groups."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xrs_amd  # noqa: E402

D, P, S, N = 12, 4, 4096, 65536


def main():
    s = torch.cuda.current_stream().cuda_stream
    x = xrs_amd.XRS(D, P)
    nbytes = N * (D + P) * S

    def group(buf, reps=10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            x.encode_batched(buf.data_ptr(), S, S, (D + P) * S, N, s)
        b.record()
        b.synchronize()
        return a.elapsed_time(b) / reps

    def report(tag, ms):
        print(json.dumps({"phase": tag, "ms": [round(m, 4) for m in ms],
                          "frac_of_8TBs": round(nbytes / float(np.median(ms)) / 1e6 / 8000, 4)}),
              flush=True)

    A = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    report("A_first", [group(A) for _ in range(5)])
    t0 = time.time()
    while time.time() - t0 < 3:
        group(A)
    report("A_after_3s", [group(A) for _ in range(5)])
    B = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda")
    ra, rb = [], []
    for _ in range(5):
        ra.append(group(A))
        rb.append(group(B))
    report("A_interleaved", ra)
    report("B_interleaved", rb)
    del A
    C = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda")
    report("C_after_free", [group(C) for _ in range(5)])


if __name__ == "__main__":
    main()
