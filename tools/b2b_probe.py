#!/usr/bin/env python3
"""Why does back-to-back 12+4 Encode @ 4 KiB (tools/refbench.py, bench_configs)
time slower than the same launch inside bench.py's step?  Per-launch HIP-event
times of Encode @ 4 KiB x 65,536 stripes when it is:
  b2b   launched back to back;
  alt   alternated with ReconstOne of the same stripes (bench.py's order);
  idle  preceded by a device synchronize and a 2 ms host sleep;
  read  preceded by a read-only pass (torch sum over an unrelated 4 GiB buffer)."""
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
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    x = xrs_amd.XRS(D, P)
    t = torch.randint(0, 256, (N * (D + P) * S,), dtype=torch.uint8, device=dev)
    other = torch.randint(0, 256, (4 << 30,), dtype=torch.uint8, device=dev).view(torch.int64)
    enc = lambda: x.encode_batched(t.data_ptr(), S, S, (D + P) * S, N, s)
    rec = lambda i: x.reconst_one_batched(t.data_ptr(), S, S, (D + P) * S, N, i % D, s)
    nbytes = N * (D + P) * S

    def measure(pre, reps=20):
        ms = []
        for i in range(reps + 2):
            pre(i)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            enc()
            b.record()
            if i >= 2:
                ms.append((a, b))
        torch.cuda.synchronize()
        v = [a.elapsed_time(b) for a, b in ms]
        return float(np.median(v))

    def idle(i):
        torch.cuda.synchronize()
        time.sleep(0.002)

    pres = {"b2b": lambda i: None, "alt": rec, "idle": idle,
            "read": lambda i: other.sum()}
    res = {k: [] for k in pres}
    for _ in range(3):
        for k, pre in pres.items():
            res[k].append(measure(pre))
    for k, v in res.items():
        ms = float(np.median(v))
        print(json.dumps({"pattern": k, "ms": round(ms, 4),
                          "gbs": round(nbytes / ms / 1e6, 1),
                          "frac_of_8TBs": round(nbytes / ms / 1e6 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
