#!/usr/bin/env python3
"""Product Encode / ReconstOne / 2-lost Reconst throughput vs the shard stride of
the batch layout, at odd vect sizes and their aligned neighbours (the
rates move with the stride through the HBM address mapping; this picks the
library's recommended strides, xrs_batch_strides).  One JSON line per case."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xrs_amd  # noqa: E402

D, P = 12, 4
CASES = {
    4096: [4096, 4112, 4160, 4224],
    4100: [4100, 4108, 4112, 4116, 4160, 4224, 8192],
    4098: [4098, 4100, 4104, 4112, 4116],
    8200: [8200, 8208, 8216, 8320],
    65538: [65538, 65552, 65600],
    1 << 20: [1 << 20, (1 << 20) + 16, (1 << 20) + 128],
    (1 << 20) + 2: [(1 << 20) + 2, (1 << 20) + 16, (1 << 20) + 32, (1 << 20) + 128],
}
ONLY = [int(v) for v in os.environ.get("SIZES", "").split(",") if v]


def timed(fn, reps=10):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.2:
        fn()
        torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps / 1e3


def main():
    x = xrs_amd.XRS(D, P)
    s = torch.cuda.current_stream().cuda_stream
    for size, strides in CASES.items():
        if ONLY and size not in ONLY:
            continue
        for shard in strides:
            stripe = (D + P) * shard
            n = (4 << 30) // stripe
            buf = torch.randint(0, 256, (n * stripe,), dtype=torch.uint8, device="cuda")
            base = buf.data_ptr()
            row = {"vect_bytes": size, "shard_stride": shard,
                   "recommended": xrs_amd.batch_strides(size, D + P)[0] == shard}
            for op, nbytes, fn in (
                    ("encode", 16 * size * n, lambda: x.encode_batched(base, size, shard, stripe, n, s)),
                    ("reconst_one", 9 * size * n,
                     lambda: x.reconst_one_batched(base, size, shard, stripe, n, 3, s)),
                    ("reconst_2", 14 * size * n,
                     lambda: x.reconst_batched(base, size, shard, stripe, n, list(range(2, 16)),
                                               [0, 1], s))):
                row[op] = round(nbytes / min(timed(fn) for _ in range(2)) / 1e9, 1)
            print(json.dumps(row), flush=True)
            del buf
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
