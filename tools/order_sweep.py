#!/usr/bin/env python3
"""Sweep XRS_BLOCK_ORDER over the four headline launches through the product
launchers (interleaved rounds, median per K).  Prints one JSON line per
(launch, K); "default" is the library's own choice.  CASES=staged sweeps the
staged general-Reconst kernel instead (2 and 4 lost data vects; GB/s of the
bytes it moves, side effects included: 16.5*S and 17.5*S per stripe)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xrs_amd  # noqa: E402

D, P = (int(v) for v in os.environ.get("CODEC", "12,4").split(","))
ROUNDS = int(os.environ.get("ROUNDS", "11"))
ORDERS = [None, "0", "16", "32", "64", "128", "256", "1024", "full"]


def time_ms(fn, reps=4):
    fn()
    torch.cuda.synchronize()
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
    cases = []
    staged = os.environ.get("CASES") == "staged"
    sizes = ((4096, 65536), (1 << 20, 512))
    if os.environ.get("SIZES"):  # e.g. SIZES=4128,8192: batches of ~4 GiB
        sizes = tuple((int(v), (4 << 30) // ((D + P) * int(v))) for v in os.environ["SIZES"].split(","))
    if os.environ.get("CASES") == "staged":
        sizes = ((4096, 65536), (64 << 10, 4096), (1 << 20, 256), (8 << 20, 32))
    for size, n in sizes:
        if staged:
            shard, stripe = xrs_amd.batch_strides(size, D + P)
            buf = torch.randint(0, 256, (n * stripe,), dtype=torch.uint8, device="cuda")
            for lost, moved in ((2, 16.5), (4, 17.5)):
                cases.append((f"reconst_{lost}_{size}", int(moved * size * n), buf,
                              lambda b=buf.data_ptr(), sz=size, sh=shard, st=stripe, nn=n,
                              lo=lost: x.reconst_batched(b, sz, sh, st, nn,
                                                         list(range(lo, D + P)),
                                                         list(range(lo)), s)))
            continue
        shard, stripe = xrs_amd.batch_strides(size, D + P)
        off = 0
        if os.environ.get("LAYOUT") == "packed":  # shards back to back at any size
            shard, stripe = size, (D + P) * size
        if os.environ.get("LAYOUT") == "layout":  # xrs_batch_layout: strides + base offset
            shard, stripe, off = xrs_amd.batch_layout(size, D + P)
        buf = torch.randint(0, 256, (n * stripe + 16,), dtype=torch.uint8, device="cuda")
        base = buf.data_ptr() + off
        cases.append((f"encode_{size}", (D + P) * size * n, buf,
                      lambda b=base, sz=size, sh=shard, st=stripe, nn=n:
                      x.encode_batched(b, sz, sh, st, nn, s)))
        a_need, _ = x.get_need_vects(3)
        cases.append((f"reconst_one_{size}", ((D + 1 + len(a_need)) * size // 2 + size) * n, buf,
                      lambda b=base, sz=size, sh=shard, st=stripe, nn=n:
                      x.reconst_one_batched(b, sz, sh, st, nn, 3, s)))
    t = {(c[0], o): [] for c in cases for o in ORDERS}
    for _ in range(ROUNDS):
        for name, _, _, fn in cases:
            for o in ORDERS:
                if o is None:
                    os.environ.pop("XRS_BLOCK_ORDER", None)
                else:
                    os.environ["XRS_BLOCK_ORDER"] = o
                t[(name, o)].append(time_ms(fn))
    os.environ.pop("XRS_BLOCK_ORDER", None)
    for name, nbytes, _, _ in cases:
        for o in ORDERS:
            med = sorted(t[(name, o)])[ROUNDS // 2]
            print(json.dumps({"launch": name, "order": o or "default",
                              "gbs": round(nbytes / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
