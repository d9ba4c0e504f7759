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
    lost2 = [0, 13]  # Reconst of one data + one piggybacked parity vect, both needed
    has2 = [j for j in range(D + P) if j not in lost2]
    fn = ((lambda i: x.encode_host(ptr, size, size, stripe, n)) if op == "encode" else
          (lambda i: x.reconst_host(ptr, size, size, stripe, n, has2, lost2))
          if op == "reconst_2" else
          (lambda i: x.reconst_one_host(ptr, size, size, stripe, n, i % D)))
    fn(0)
    t0 = time.perf_counter()
    for i in range(reps):
        fn(i)
    dt = (time.perf_counter() - t0) / reps
    # reconst_2: accounted (d + lost) * S (xrs_test.go:565); 14 survivors up,
    # lost a-halves + needed b-halves + retrieveRS b-halves (14, 15) back
    algo = n * {"encode": 16, "reconst_one": 9, "reconst_2": D + 2}[op] * size
    h2d = n * {"encode": D, "reconst_one": 8, "reconst_2": D + P - 2}[op] * size
    d2h = n * {"encode": P, "reconst_one": 1, "reconst_2": 3}[op] * size
    if pinned:
        xrs_amd.lib().xrs_host_free(ptr)
    return {"op": op, "vect_bytes": size, "stripes": n, "pinned": pinned,
            "ms": round(dt * 1e3, 3), "algorithmic_gibps": round(algo / dt / 2**30, 2),
            "h2d_gbs": round(h2d / dt / 1e9, 2), "d2h_gbs": round(d2h / dt / 1e9, 2)}


def run_zero_copy(op, size, n, reps):
    """The *_batched kernels run directly on pinned, mapped host memory (no
    DMA): reads and writes cross PCIe from the kernel.  Parity is checked
    against the oracle on the first stripes."""
    import torch
    from oracle.oracle_c import OracleXRS
    stripe = 16 * size
    ptr, buf = host_buf(n * stripe, True)
    dptr = xrs_amd.lib().xrs_host_device_pointer(ptr)
    assert dptr, "no device mapping"
    buf[:] = np.random.default_rng(3).integers(0, 256, size=n * stripe, dtype=np.uint8)
    x = xrs_amd.XRS(D, P)
    x.encode_batched(dptr, size, size, stripe, n, 0)
    torch.cuda.synchronize()
    o = OracleXRS(D, P)
    for s in range(min(n, 4)):
        v = [buf[s * stripe + i * size: s * stripe + (i + 1) * size].copy() for i in range(16)]
        w = [r.copy() for r in v]
        o.encode(w)
        assert all(np.array_equal(a, b) for a, b in zip(v, w)), s
    fn = ((lambda i: x.encode_batched(dptr, size, size, stripe, n, 0)) if op == "encode" else
          (lambda i: x.reconst_one_batched(dptr, size, size, stripe, n, i % D, 0)))
    fn(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        fn(i)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    # reconst_2: accounted (d + lost) * S (xrs_test.go:565); 14 survivors up,
    # lost a-halves + needed b-halves + retrieveRS b-halves (14, 15) back
    algo = n * {"encode": 16, "reconst_one": 9, "reconst_2": D + 2}[op] * size
    h2d = n * {"encode": D, "reconst_one": 8, "reconst_2": D + P - 2}[op] * size
    d2h = n * {"encode": P, "reconst_one": 1, "reconst_2": 3}[op] * size
    xrs_amd.lib().xrs_host_free(ptr)
    return {"op": op, "vect_bytes": size, "stripes": n, "pinned": True, "mode": "zero-copy kernel",
            "ms": round(dt * 1e3, 3), "algorithmic_gibps": round(algo / dt / 2**30, 2),
            "h2d_gbs": round(h2d / dt / 1e9, 2), "d2h_gbs": round(d2h / dt / 1e9, 2)}


def run_group(op, size, n, devices, reps):
    """xrs_group_*: the host batch split across `devices` (one PCIe link each),
    pinned memory, kernels in place."""
    stripe = 16 * size
    ptr, buf = host_buf(n * stripe, True)
    buf[:] = np.random.default_rng(3).integers(0, 256, size=n * stripe, dtype=np.uint8)
    g = xrs_amd.XRSGroup(D, P, devices)
    g.encode_host(ptr, size, size, stripe, n)
    fn = ((lambda i: g.encode_host(ptr, size, size, stripe, n)) if op == "encode" else
          (lambda i: g.reconst_one_host(ptr, size, size, stripe, n, i % D)))
    fn(0)
    t0 = time.perf_counter()
    for i in range(reps):
        fn(i)
    dt = (time.perf_counter() - t0) / reps
    algo = n * (16 if op == "encode" else 9) * size
    del g
    xrs_amd.lib().xrs_host_free(ptr)
    return {"op": op, "vect_bytes": size, "stripes": n, "pinned": True,
            "mode": f"group of {len(devices)} GPU(s) {devices}", "ms": round(dt * 1e3, 3),
            "algorithmic_gibps": round(algo / dt / 2**30, 2)}


def main():
    cases = [("encode", 4096, 16384), ("encode", 1 << 20, 64),
             ("reconst_one", 1 << 20, 64), ("reconst_one", 4096, 16384),
             ("reconst_2", 4096, 16384), ("reconst_2", 1 << 20, 64)]
    modes = sys.argv[1:] or ["pipeline", "zero-copy"]
    if "reconst2" in modes:  # only the general-Reconst rows, pipeline modes
        cases, modes = [c for c in cases if c[0] == "reconst_2"], ["pipeline"]
    if "odd" in modes:  # odd vect sizes (back-to-back shards), pipeline modes
        cases = [("encode", 4098, 16384), ("encode", 4100, 16384), ("encode", (1 << 20) + 2, 64),
                 ("reconst_one", 4098, 16384), ("reconst_one", (1 << 20) + 2, 64)]
        modes = ["pipeline"]
    for op, size, n in cases:
        if "pipeline" in modes:
            for pinned, zc in ((True, "1"), (True, "0"), (False, "0")):
                os.environ["XRS_HOST_ZC"] = zc  # pinned: in place (1) or copy pipeline (0)
                r = run(op, size, n, pinned, reps=5 if pinned else 2)
                r["mode"] = "in place (zero copy)" if pinned and zc == "1" else "copy pipeline"
                print(json.dumps(r), flush=True)
            os.environ.pop("XRS_HOST_ZC", None)
        if "zero-copy" in modes and op != "reconst_2":
            print(json.dumps(run_zero_copy(op, size, n, reps=5)), flush=True)
        if "group" in modes and op != "reconst_2":
            import torch
            ndev = torch.cuda.device_count()
            for devs in ([0], list(range(ndev))) if ndev > 1 else ([0],):
                print(json.dumps(run_group(op, size, n * len(devs), devs, reps=5)), flush=True)


if __name__ == "__main__":
    main()
