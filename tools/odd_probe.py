#!/usr/bin/env python3
"""Throughput of the byte-granular kernels (half-vect not a multiple of 16 B,
or rows not 16-B aligned) against the 16-B kernels: Encode / ReconstOne /
Update of 12+4 stripes near 4 KiB and 1 MiB."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xrs_amd  # noqa: E402

D, P = 12, 4


def timed(fn, reps=10):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        fn()
        torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps / 1e3


# (env var, value) pairs A/B'd: the ragged end in the 16-B launch (default) or
# its own launch.  (Padding each stripe's lanes to whole waves, so no wave
# spans two stripes, measured 0-10% slower: profiles/r02_odd_probe2.log.)
TAILS = {"overlap": {}, "launch": {"XRS_TAIL": "launch"}}


def main():
    x = xrs_amd.XRS(D, P)
    s = torch.cuda.current_stream().cuda_stream
    for size, n, base_off in ((4096, 65536, 0), (4128, 65536, 0), (4100, 65536, 0), (4098, 65536, 0),
                              (4096, 65536, 4), (1 << 20, 256, 0), ((1 << 20) + 2, 256, 0)):
        stripe = (D + P) * size
        buf = torch.randint(0, 256, (n * stripe + 64,), dtype=torch.uint8, device="cuda")
        base = buf.data_ptr() + base_off
        for op, nbytes, fn in (
                ("encode", 16 * size * n, lambda: x.encode_batched(base, size, size, stripe, n, s)),
                ("reconst_one", 9 * size * n,
                 lambda: x.reconst_one_batched(base, size, size, stripe, n, 3, s))):
            best = {}
            for rep in range(3):  # interleaved A/B rounds; best of each
                for tail, env in TAILS.items():
                    os.environ.pop("XRS_TAIL", None)
                    os.environ.update(env)
                    secs = timed(fn)
                    best[tail] = min(best.get(tail, 1e9), secs)
            os.environ.pop("XRS_TAIL", None)
            print(json.dumps({"op": op, "vect_bytes": size, "base_off": base_off,
                              **{f"gbs_{t}": round(nbytes / best[t] / 1e9, 1) for t in TAILS}}),
                  flush=True)
        del buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
