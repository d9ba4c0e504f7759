#!/usr/bin/env python3
"""End-to-end (PCIe-inclusive) rates of the host-resident pipelined path:
shards start and end in host memory (north_star: "the end-to-end rate including
pinned hipMemcpyAsync in and out is also measured and written in DESIGN.md").

Prints one JSON line per configuration (not the driver's bench contract).
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xrs_amd  # noqa: E402

D, P = 12, 4


def host_buf(nbytes, pinned):
    if pinned:
        p = xrs_amd.lib().xrs_host_alloc(nbytes)
        assert p, "pinned alloc failed"
        return p, np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))
    a = np.empty(nbytes, np.uint8)
    return a.ctypes.data, a


def run(op, size, n, pinned, reps):
    stripe = 16 * size
    ptr, buf = host_buf(n * stripe, pinned)
    buf[:] = np.random.default_rng(3).integers(0, 256, size=n * stripe, dtype=np.uint8)
    x = xrs_amd.XRS(D, P)
    x.encode_host(ptr, size, size, stripe, n)  # warm + valid stripes
    fn = ((lambda i: x.encode_host(ptr, size, size, stripe, n)) if op == "encode" else
          (lambda i: x.reconst_one_host(ptr, size, size, stripe, n, i % D)))
    fn(0)
    t0 = time.perf_counter()
    for i in range(reps):
        fn(i)
    dt = (time.perf_counter() - t0) / reps
    algo = n * (16 if op == "encode" else 9) * size
    h2d = n * (D if op == "encode" else 8) * size
    d2h = n * (P if op == "encode" else 1) * size
    if pinned:
        xrs_amd.lib().xrs_host_free(ptr)
    return {"op": op, "vect_bytes": size, "stripes": n, "pinned": pinned,
            "ms": round(dt * 1e3, 3), "algorithmic_gibps": round(algo / dt / 2**30, 2),
            "h2d_gbs": round(h2d / dt / 1e9, 2), "d2h_gbs": round(d2h / dt / 1e9, 2)}


def main():
    for op, size, n in [("encode", 4096, 16384), ("encode", 1 << 20, 64),
                        ("reconst_one", 1 << 20, 64), ("reconst_one", 4096, 16384)]:
        for pinned in (True, False):
            print(json.dumps(run(op, size, n, pinned, reps=5 if pinned else 2)), flush=True)


if __name__ == "__main__":
    main()
