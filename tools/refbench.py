#!/usr/bin/env python3
"""The reference's own benchmark matrix on one MI355X, device-resident.

One JSON line per sub-benchmark of /root/reference/xrs_test.go, named as `go
test -bench` names it, with the reference's SetBytes accounting:

  * BenchmarkXRS_Encode  (:471-521)  12+4 @ 4 KiB, 1 MiB, 8 MiB   (d+p)*S
  * BenchmarkXRS_Reconst (:523-582)  12+4 @ 4 KiB, lost data[:i], i = 1..4
                                     i = 1: (d-1+2+|aNeed|)*S/2 + S, else (d+i)*S
  * BenchmarkXRS_Update  (:584-630)  12+4 @ 4 KiB                  (2p+2)*S
  * BenchmarkXRS_Replace (:632-680)  12+4 @ 4 KiB, rows[:n], n = 1..8  (n+2p)*S

The Go benchmark loops one stripe b.N times; here one launch covers a batch
of stripes (>= 2 GiB of algorithmic bytes, so nothing is served from the
256 MiB Infinity Cache), and the line reports the batch rate and the
reference's published single-core figure for the same row (README.md:80-118,
i7-7700HQ).  The per-stripe synchronous calls of the same rows are timed by
tools/sync_bench (`ref` mode).
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xrs_amd  # noqa: E402

D, P = 12, 4
KB, MB = 1 << 10, 1 << 20
PEAK = 8.0e12
# README.md:80-118 (MB/s = 1e6 B/s, one i7-7700HQ core).
README_MBS = {
    "Encode/(12+4)-4KB": 10895.15, "Encode/(12+4)-1MB": 7530.84, "Encode/(12+4)-8MB": 6579.53,
    "Reconst/(12+4)-4KB-reconst_1_data_vects": 10334.99, "Reconst/(12+4)-4KB-reconst_2_data_vects": 9654.17,
    "Reconst/(12+4)-4KB-reconst_3_data_vects": 8164.76, "Reconst/(12+4)-4KB-reconst_4_data_vects": 7404.41,
    "Update/(12+4)-4KB": 26312.14,
    "Replace/(12+4)-4KB-replace_1_data_vects": 44082.57, "Replace/(12+4)-4KB-replace_2_data_vects": 26554.30,
    "Replace/(12+4)-4KB-replace_3_data_vects": 19583.16, "Replace/(12+4)-4KB-replace_4_data_vects": 16636.82,
    "Replace/(12+4)-4KB-replace_5_data_vects": 14301.15, "Replace/(12+4)-4KB-replace_6_data_vects": 13121.98,
    "Replace/(12+4)-4KB-replace_7_data_vects": 12028.10, "Replace/(12+4)-4KB-replace_8_data_vects": 11300.55,
}


def size_str(n):  # byteToStr, xrs_test.go:682
    return f"{n // MB}MB" if n >= MB else f"{n // KB}KB"


def timed(fn, reps=10, warm=2, ramp=0.3):
    # An idle GPU runs its first launches slowly (profiles/r01_first_alloc.log):
    # warm for `ramp` seconds as well as `warm` launches.
    t0, i = time.perf_counter(), 0
    while i < warm or time.perf_counter() - t0 < ramp:
        fn(i)
        torch.cuda.synchronize()
        i += 1
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for i in range(reps):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps / 1e3


def emit(bench, name, size, n, secs, bytes_per_stripe):
    total = n * bytes_per_stripe
    ref = README_MBS.get(bench.replace("BenchmarkXRS_", "") + "/" + name)
    rate = total / secs
    print(json.dumps({
        "bench": f"{bench}/{name}", "vect_bytes": size, "stripes": n,
        "bytes_per_stripe": bytes_per_stripe, "ms": round(secs * 1e3, 4),
        "MB_s": round(rate / 1e6, 1), "gibps": round(rate / 2**30, 1),
        "frac_of_8TBs": round(rate / PEAK, 4), "ns_per_stripe": round(secs / n * 1e9, 2),
        "readme_i7_1core_MB_s": ref, "x_readme": round(rate / 1e6 / ref, 1) if ref else None,
    }), flush=True)


def stripes_for(bytes_per_stripe, floor=2 << 30):
    n = 1
    while n * bytes_per_stripe < floor:
        n *= 2
    return n


def main():
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    x = xrs_amd.XRS(D, P)

    def batch(size, n, seed):
        shard, stripe = xrs_amd.batch_strides(size, D + P)
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        t = torch.randint(0, 256, (n * stripe,), dtype=torch.uint8, device=dev, generator=g)
        return t, shard, stripe

    # BenchmarkXRS_Encode
    for size in (4 * KB, MB, 8 * MB):
        n = stripes_for((D + P) * size, 4 << 30)
        t, sh, st = batch(size, n, 1)
        secs = timed(lambda i: x.encode_batched(t.data_ptr(), size, sh, st, n, s))
        emit("BenchmarkXRS_Encode", f"(12+4)-{size_str(size)}", size, n, secs, (D + P) * size)
        del t

    size = 4 * KB
    n = 65536  # 4 GiB of stripes
    t, sh, st = batch(size, n, 2)
    x.encode_batched(t.data_ptr(), size, sh, st, n, s)
    # BenchmarkXRS_Reconst: lost = data[:i], dpHas = the rest (makeHasFromLost)
    for i in range(1, P + 1):
        lost = list(range(i))
        has = list(range(i, D + P))
        if i == 1:
            a_need, _ = x.get_need_vects(0)
            bps = (D - 1 + 2 + len(a_need)) * size // 2 + size
        else:
            bps = (D + i) * size
        secs = timed(lambda j: x.reconst_batched(t.data_ptr(), size, sh, st, n, has, lost, s))
        emit("BenchmarkXRS_Reconst", f"(12+4)-4KB-reconst_{i}_data_vects", size, n,
             secs, bps)
    # BenchmarkXRS_Update: vects[row] -> newData, parity vects[d:]
    row = 5
    new = torch.randint(0, 256, (n * size,), dtype=torch.uint8, device=dev)
    par = t.data_ptr() + D * sh
    secs = timed(lambda j: x.update_batched(t.data_ptr() + row * sh, st, new.data_ptr(), size,
                                            size, row, par, sh, st, n, s))
    emit("BenchmarkXRS_Update", "(12+4)-4KB", size, n, secs, (2 * P + 2) * size)
    del new
    # BenchmarkXRS_Replace: data vects[:n] at rows 0..n-1, parity vects[d:]
    for k in range(1, D - P + 1):
        rows = list(range(k))
        secs = timed(lambda j: x.replace_batched(t.data_ptr(), sh, st, rows, size, par, sh, st, n,
                                                 s))
        emit("BenchmarkXRS_Replace", f"(12+4)-4KB-replace_{k}_data_vects", size, n, secs,
             (k + 2 * P) * size)
    del t
    torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
