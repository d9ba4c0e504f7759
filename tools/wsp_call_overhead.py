#!/usr/bin/env python3
"""Wall time per synchronous 2-lost Reconst call (launch + wait) for a few
batch sizes at 1 MiB vects: the persistent kernel forced (XRS_WSP=512; its
per-launch counter: stream-ordered alloc + memset + free) and the default
against the one-shot kernel (XRS_WSP=0), interleaved.  Timing only."""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xrs_amd  # noqa: E402


def main():
    x = xrs_amd.XRS(12, 4)
    s = torch.cuda.current_stream().cuda_stream
    S = 1 << 20
    has = list(range(2, 16))
    for n in (1, 4, 16, 64, 128, 256):
        buf = torch.randint(0, 256, (n * 16 * S,), dtype=torch.uint8, device="cuda")
        res = {"0": [], "512": [], "": []}
        for r in range(7):
            for v in ("0", "512", ""):
                os.environ["XRS_WSP"] = v
                for _ in range(3):
                    x.reconst_batched(buf.data_ptr(), S, S, 16 * S, n, has, [0, 1], s)
                torch.cuda.synchronize()
                k = 20
                t0 = time.perf_counter()
                for _ in range(k):
                    x.reconst_batched(buf.data_ptr(), S, S, 16 * S, n, has, [0, 1], s)
                    torch.cuda.synchronize()
                res[v].append((time.perf_counter() - t0) / k * 1e6)
        print(f"n={n:4d} stripes of 1 MiB: one-shot {statistics.median(res['0']):8.1f} us/call, "
              f"persistent {statistics.median(res['512']):8.1f}, default {statistics.median(res['']):8.1f}",
              flush=True)
        del buf


if __name__ == "__main__":
    main()
