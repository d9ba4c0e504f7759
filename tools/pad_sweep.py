#!/usr/bin/env python3
"""Shard-stride padding sweep at 1 MiB (and 8 MiB) vects, in the kernels'
XCD block order: Encode and ReconstOne of 12+4 stripes with shard stride
S + pad for several pads (interleaved rounds, median).  GB/s of algorithmic
bytes.  Informs xrs_batch_strides' recommended layout."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xrs_amd  # noqa: E402

D, P = 12, 4
PADS = [0, 256, 1024, 2048, 4096, 4096 + 256, 8192, 65536]
ROUNDS = int(os.environ.get("ROUNDS", "7"))


def time_ms(fn, reps=4):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def main():
    x = xrs_amd.XRS(D, P)
    s = torch.cuda.current_stream().cuda_stream
    for size, n in ((1 << 20, 512), (8 << 20, 64)):
        maxstride = (D + P) * (size + max(PADS))
        buf = torch.randint(0, 256, (n * maxstride,), dtype=torch.uint8, device="cuda")
        for _ in range(50):  # clock ramp
            x.encode_batched(buf.data_ptr(), size, size, (D + P) * size, n, s)
        torch.cuda.synchronize()
        res = {(op, pad): [] for op in ("encode", "reconst_one") for pad in PADS}
        for _ in range(ROUNDS):
            for pad in PADS:
                sh = size + pad
                st = (D + P) * sh
                res[("encode", pad)].append(
                    time_ms(lambda: x.encode_batched(buf.data_ptr(), size, sh, st, n, s)))
                res[("reconst_one", pad)].append(
                    time_ms(lambda: x.reconst_one_batched(buf.data_ptr(), size, sh, st, n, 3, s)))
        for (op, pad), v in res.items():
            med = sorted(v)[ROUNDS // 2]
            nbytes = n * size * (16 if op == "encode" else 9)
            print(json.dumps({"op": op, "vect_bytes": size, "pad": pad,
                              "gbs": round(nbytes / med / 1e6, 1)}), flush=True)
        del buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
