#!/usr/bin/env python3
"""Interleaved A/B of one launch-time environment knob through the product
launchers: VAR=XRS_PAIR_BLOCK VALS=256,128 CASE=encode SIZE=1048576 [CODEC=12,4]
[ROUNDS=15] [STRIPES=n, default ~4 GiB of vects].  CASE is encode, reconst_one, reconst_2 / _3 / _4 (lost data
vects, staged path), update or replace_K.  One JSON line per value: median GB/s of the bytes the launch
moves (rounds alternate the values, so box drift hits both alike)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xrs_amd  # noqa: E402


def main():
    d, p = (int(v) for v in os.environ.get("CODEC", "12,4").split(","))
    var = os.environ["VAR"]
    vals = os.environ["VALS"].split(",")
    case = os.environ.get("CASE", "encode")
    size = int(os.environ.get("SIZE", str(1 << 20)))
    rounds = int(os.environ.get("ROUNDS", "15"))
    n = int(os.environ.get("STRIPES", "0")) or (4 << 30) // ((d + p) * size)
    x = xrs_amd.XRS(d, p)
    s = torch.cuda.current_stream().cuda_stream
    shard, stripe = xrs_amd.batch_strides(size, d + p)
    buf = torch.randint(0, 256, (n * stripe,), dtype=torch.uint8, device="cuda")
    b = buf.data_ptr()
    if case == "encode":
        moved = (d + p) * size * n
        fn = lambda: x.encode_batched(b, size, shard, stripe, n, s)  # noqa: E731
    elif case == "reconst_one":
        a_need, _ = x.get_need_vects(3)
        moved = ((d + 1 + len(a_need)) * size // 2 + size) * n
        fn = lambda: x.reconst_one_batched(b, size, shard, stripe, n, 3, s)  # noqa: E731
    elif case in ("reconst_2", "reconst_3", "reconst_4"):
        lost = int(case[-1])  # bytes moved at 12+4, side effects included (else accounted)
        moved = int({2: 16.5, 3: 17.0, 4: 17.5}[lost] * size * n) if (d, p) == (12, 4) \
            else (d + lost) * size * n
        fn = lambda: x.reconst_batched(b, size, shard, stripe, n,  # noqa: E731
                                       list(range(lost, d + p)), list(range(lost)), s)
    elif case.startswith("mixed_"):  # mixed_0-13: those vects lost and needed, (d + lost) * S
        lost = [int(v) for v in case.split("_")[1].split("-")]
        has = [i for i in range(d + p) if i not in lost]
        moved = (d + len(lost)) * size * n
        fn = lambda: x.reconst_batched(b, size, shard, stripe, n, has, lost, s)  # noqa: E731
    elif case == "update":  # one data row (3) of every stripe, new bytes back to back
        new = torch.randint(0, 256, (n * size,), dtype=torch.uint8, device="cuda")
        moved = (2 * p + 2) * size * n
        fn = lambda: x.update_batched(b + 3 * shard, stripe, new.data_ptr(), size,  # noqa: E731
                                      size, 3, b + d * shard, shard, stripe, n, s)
    elif case.startswith("replace_"):  # Replace(k): data rows 0..k-1
        k = int(case.split("_")[1])
        moved = (k + 2 * p) * size * n
        fn = lambda: x.replace_batched(b, shard, stripe, list(range(k)), size,  # noqa: E731
                                       b + d * shard, shard, stripe, n, s)
    else:
        raise SystemExit(f"unknown CASE {case}")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t = {v: [] for v in vals}
    # VAR=MULTI: each value sets several variables, "K1=V1+K2=V2" ("" = all
    # of them unset); every variable any value names is unset first
    multi_keys = sorted({kv.split("=")[0] for v in vals for kv in v.split("+") if kv}) \
        if var == "MULTI" else []
    for _ in range(rounds):
        for v in vals:
            if var == "MULTI":
                for k in multi_keys:
                    os.environ.pop(k, None)
                for kv in (v.split("+") if v else []):
                    k, _, val = kv.partition("=")
                    os.environ[k] = val
            elif v:
                os.environ[var] = v
            else:  # an empty value = the library's default (variable unset)
                os.environ.pop(var, None)
            fn()
            ev[0].record()
            for _ in range(4):
                fn()
            ev[1].record()
            ev[1].synchronize()
            t[v].append(ev[0].elapsed_time(ev[1]) / 4)
    for v in vals:
        med = sorted(t[v])[rounds // 2]
        print(json.dumps({"var": var, "val": v, "case": case, "size": size, "codec": f"{d}+{p}",
                          "ms": round(med, 4), "gbs": round(moved / med / 1e6, 1)}))


if __name__ == "__main__":
    main()
