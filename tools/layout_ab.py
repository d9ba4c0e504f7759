#!/usr/bin/env python3
"""Interleaved A/B of batch layouts (shard stride, stripe stride) for one
launch: CODEC=12,3 SIZE=4096 CASE=reconst_one LAYOUTS=4096:61440,4096:65536
[ROUNDS=15] [GIB=4].  A layout entry "shard:stripe" in bytes ("rec" = the
library's recommendation; "sm" or "sm:PAD" = shard-major, each shard's
rows back to back over the stripes: stripe stride = size, shard stride =
n*size + PAD).  One JSON line per layout: median GB/s of the
bytes the launch moves."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xrs_amd  # noqa: E402


def main():
    d, p = (int(v) for v in os.environ.get("CODEC", "12,3").split(","))
    case = os.environ.get("CASE", "reconst_one")
    size = int(os.environ.get("SIZE", "4096"))
    rounds = int(os.environ.get("ROUNDS", "15"))
    gib = float(os.environ.get("GIB", "4"))
    n = int(gib * (1 << 30)) // ((d + p) * size)
    x = xrs_amd.XRS(d, p)
    s = torch.cuda.current_stream().cuda_stream
    layouts = []
    for e in os.environ.get("LAYOUTS", "rec").split(","):
        if e == "rec":
            layouts.append(("rec",) + tuple(xrs_amd.batch_strides(size, d + p)))
        elif e.startswith("sm"):
            pad = int(e[3:] or 0) if ":" in e else 0
            layouts.append((e, n * size + pad, size))
        else:  # "shard:stripe" or "shard:stripe@offset" (batch base + offset bytes)
            lay, _, o = e.partition("@")
            sh, st = (int(v) for v in lay.split(":"))
            assert sh >= size and st >= (d + p) * sh
            layouts.append((e, sh, st))
    offs = {name: int(name.partition("@")[2] or 0) for name, _, _ in layouts}
    extent = max((n - 1) * st + (d + p - 1) * sh + size + offs[nm] for nm, sh, st in layouts)
    buf = torch.randint(0, 256, (extent,), dtype=torch.uint8, device="cuda")
    b0 = buf.data_ptr()
    assert b0 % 4096 == 0
    a_need, _ = x.get_need_vects(3)
    # reconst_L: L lost data vects (staged kernel); bytes it moves at 12+4,
    # side effects included (tools/order_sweep.py): 16.5 / 17.5 S at 2 / 4
    moved = {"encode": (d + p) * size * n,
             "reconst_one": ((d + 1 + len(a_need)) * size // 2 + size) * n,
             "reconst_2": int(16.5 * size * n), "reconst_4": int(17.5 * size * n)}[case]

    def fn(sh, st, b):
        if case == "encode":
            x.encode_batched(b, size, sh, st, n, s)
        elif case == "reconst_one":
            x.reconst_one_batched(b, size, sh, st, n, 3, s)
        else:
            lost = int(case[-1])
            x.reconst_batched(b, size, sh, st, n, list(range(lost, d + p)), list(range(lost)), s)

    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t = {name: [] for name, _, _ in layouts}
    for _ in range(rounds):
        for name, sh, st in layouts:
            fn(sh, st, b0 + offs[name])
            ev[0].record()
            for _ in range(4):
                fn(sh, st, b0 + offs[name])
            ev[1].record()
            ev[1].synchronize()
            t[name].append(ev[0].elapsed_time(ev[1]) / 4)
    for name, sh, st in layouts:
        med = sorted(t[name])[rounds // 2]
        print(json.dumps({"layout": name, "shard_stride": sh, "stripe_stride": st, "case": case,
                          "size": size, "codec": f"{d}+{p}", "stripes": n, "ms": round(med, 4),
                          "gbs": round(moved / med / 1e6, 1)}))


if __name__ == "__main__":
    main()
