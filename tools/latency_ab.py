#!/usr/bin/env python3
"""A/B of the latency-bound (single-stripe) kernel loops through the sync
API: per-call time of ReconstOne / Reconst on one 4 KiB stripe for a
runtime-shaped codec with the rows kernel's grouped and row-at-a-time loops
(XRS_ROWS_GROUPED), and for 12+4 multi-loss Reconst with the staged kernel's
all-loads-first and late-b variants (XRS_STAGED_LATE).  Interleaved rounds,
medians."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xrs_amd  # noqa: E402


def per_call(fn, secs=0.3):
    fn()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < secs:
        fn()
        n += 1
    return (time.perf_counter() - t0) / n * 1e6


def main():
    rng = np.random.default_rng(1)
    size = 4096
    cases = []
    for d, p in ((10, 4), (6, 3), (20, 4)):
        x = xrs_amd.XRS(d, p)
        v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(d + p)]
        x.encode(v)
        has = list(range(2, d + p))
        cases.append((f"reconst_one_{d}+{p}", "XRS_ROWS_GROUPED", lambda x=x, v=v: x.reconst_one(v, 0)))
        cases.append((f"reconst_2_steps_{d}+{p}", "XRS_ROWS_GROUPED",
                      lambda x=x, v=v, has=has: x.reconst(v, has, [0, 1])))
    x = xrs_amd.XRS(12, 4)
    v = [rng.integers(0, 256, size=size, dtype=np.uint8) for _ in range(16)]
    x.encode(v)
    for lost in (2, 3, 4):
        has = list(range(lost, 16))
        cases.append((f"reconst_{lost}_staged_12+4", "XRS_STAGED_LATE",
                      lambda v=v, has=has, lost=lost: x.reconst(v, has, list(range(lost)))))
    for name, env, fn in cases:
        if name.startswith("reconst_2_steps"):
            os.environ["XRS_RECONST"] = "steps"
        res = {"0": [], "1": []}
        for _ in range(5):
            for val in ("0", "1"):
                os.environ[env] = val
                res[val].append(per_call(fn))
        os.environ.pop(env, None)
        os.environ.pop("XRS_RECONST", None)
        print(json.dumps({"case": name, "env": env, "us_0": round(float(np.median(res["0"])), 1),
                          "us_1": round(float(np.median(res["1"])), 1)}), flush=True)


if __name__ == "__main__":
    main()
