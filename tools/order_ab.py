#!/usr/bin/env python3
"""A/B of the XCD-aware block order through the product launchers.

For each (op, vect size, layout) case, interleaved rounds of the plain order
(XRS_BLOCK_ORDER=0) and the library's default order; median per variant.  The
two orders must write identical bytes (checked on the parity / rebuilt rows).
Prints one JSON line per case.
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xrs_amd  # noqa: E402

D, P = 12, 4
ROUNDS = 7


def time_ms(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def case(x, size, n, pad, stream):
    shard = size + pad
    stripe = 16 * shard
    buf = torch.randint(0, 256, (n * stripe,), dtype=torch.uint8, device="cuda")
    base = buf.data_ptr()
    view = buf.view(n, 16, shard)[:, :, :size]
    ops = {
        "encode": (lambda: x.encode_batched(base, size, shard, stripe, n, stream), 16 * size * n,
                   lambda: view[:, D:].clone()),
        "reconst_one": (lambda: x.reconst_one_batched(base, size, shard, stripe, n, 5, stream),
                        9 * size * n, lambda: view[:, 5].clone()),
    }
    out = []
    for op, (fn, nbytes, snap) in ops.items():
        res = {}
        for order in ("0", None):
            if order is None:
                os.environ.pop("XRS_BLOCK_ORDER", None)
            else:
                os.environ["XRS_BLOCK_ORDER"] = order
            fn()
            torch.cuda.synchronize()
            res[order] = snap()
        same = bool(torch.equal(res["0"], res[None]))
        t = {"0": [], None: []}
        for _ in range(ROUNDS):
            for order in ("0", None):
                if order is None:
                    os.environ.pop("XRS_BLOCK_ORDER", None)
                else:
                    os.environ["XRS_BLOCK_ORDER"] = order
                t[order].append(time_ms(fn))
        os.environ.pop("XRS_BLOCK_ORDER", None)
        med = {k: sorted(v)[ROUNDS // 2] for k, v in t.items()}
        out.append({"op": op, "vect_bytes": size, "stripes": n, "pad": pad, "same_bytes": same,
                    "plain_gbs": round(nbytes / med["0"] / 1e6, 1),
                    "xcd_gbs": round(nbytes / med[None] / 1e6, 1),
                    "gain": round(med["0"] / med[None], 4)})
    del buf
    torch.cuda.empty_cache()
    return out


def main():
    x = xrs_amd.XRS(D, P)
    stream = torch.cuda.current_stream().cuda_stream
    cases = [(4096, 65536, 0), (16384, 16384, 0), (65536, 4096, 0), (65536, 4096, 256),
             (1 << 20, 512, 0), (1 << 20, 512, 256), (8 << 20, 64, 0), (8 << 20, 64, 4096 + 256)]
    for size, n, pad in cases:
        for r in case(x, size, n, pad, stream):
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
