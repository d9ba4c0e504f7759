#!/usr/bin/env python3
"""Device-resident throughput of every BASELINE.json config on one MI355X
(the driver's bench.py line covers the headline; this fills DESIGN.md).

Byte accounting = the reference's SetBytes (xrs_test.go:513, :565-572, :622,
:672): Encode (d+p)*S, ReconstOne 9*S, Reconst(n lost data) (d+n)*S,
Update (2p+2)*S, Replace(n) (n+2p)*S per stripe.  One JSON line per case.
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
PEAK = 8.0e12


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


def emit(name, size, n, secs, nbytes, shard):
    print(json.dumps({"case": name, "vect_bytes": size, "stripes": n, "shard_stride": shard,
                      "ms": round(secs * 1e3, 4), "gibps": round(nbytes / secs / 2**30, 1),
                      "gbs": round(nbytes / secs / 1e9, 1),
                      "frac_of_8TBs": round(nbytes / secs / PEAK, 4)}), flush=True)


def batch(size, n, dev, seed, padded=True):
    shard, stripe = xrs_amd.batch_strides(size, D + P) if padded else (size, (D + P) * size)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    t = torch.randint(0, 256, (n * stripe,), dtype=torch.uint8, device=dev, generator=g)
    return t, shard, stripe


def main():
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    x = xrs_amd.XRS(D, P)
    cases = sys.argv[1:] or ["c2", "c3", "c4", "c5", "multi"]
    if "c2" in cases:  # 12+4 Encode @ 4 KiB
        for padded in (True, False):
            t, sh, st = batch(4096, 65536, dev, 1, padded)
            secs = timed(lambda i: x.encode_batched(t.data_ptr(), 4096, sh, st, 65536, s))
            emit("encode", 4096, 65536, secs, 65536 * 16 * 4096, sh)
            del t
    if "c3" in cases:  # ReconstOne @ 1 MiB
        for padded in (True, False):
            t, sh, st = batch(1 << 20, 512, dev, 2, padded)
            x.encode_batched(t.data_ptr(), 1 << 20, sh, st, 512, s)
            secs = timed(lambda i: x.reconst_one_batched(t.data_ptr(), 1 << 20, sh, st, 512, i % D, s))
            emit("reconst_one", 1 << 20, 512, secs, 512 * 9 * (1 << 20), sh)
            del t
    if "c4" in cases:  # Update + Replace(4) @ 8 MiB
        size, n = 8 << 20, 32
        t, sh, st = batch(size, n, dev, 3)
        x.encode_batched(t.data_ptr(), size, sh, st, n, s)
        new = torch.randint(0, 256, (n * size,), dtype=torch.uint8, device=dev)
        par = t.data_ptr() + D * sh
        secs = timed(lambda i: x.update_batched(t.data_ptr() + (i % D) * sh, st, new.data_ptr(),
                                                size, size, i % D, par, sh, st, n, s))
        emit("update", size, n, secs, n * (2 * P + 2) * size, sh)
        for nrep in (1, 4, 8):
            rows = list(range(nrep))
            secs = timed(lambda i: x.replace_batched(t.data_ptr(), sh, st, rows, size, par, sh, st,
                                                     n, s))
            emit(f"replace_{nrep}", size, n, secs, n * (nrep + 2 * P) * size, sh)
        del t, new
    if "rows" in cases:  # Update with a per-stripe random row (xrs_update_rows_batched)
        for size, n in ((4096, 65536), (1 << 20, 256)):
            t, sh, st = batch(size, n, dev, 6)
            x.encode_batched(t.data_ptr(), size, sh, st, n, s)
            new = torch.randint(0, 256, (n * size,), dtype=torch.uint8, device=dev)
            old = torch.randint(0, 256, (n * size,), dtype=torch.uint8, device=dev)
            rows = torch.randint(0, D, (n,), dtype=torch.int32, device=dev)
            par = t.data_ptr() + D * sh
            secs = timed(lambda i: x.update_rows_batched(old.data_ptr(), size, new.data_ptr(), size,
                                                         size, rows.data_ptr(), par, sh, st, n, s))
            emit("update_rows", size, n, secs, n * (2 * P + 2) * size, sh)
            secs = timed(lambda i: x.update_batched(old.data_ptr(), size, new.data_ptr(), size,
                                                    size, 5, par, sh, st, n, s))
            emit("update_one_row", size, n, secs, n * (2 * P + 2) * size, sh)
            del t, new, old, rows
    if "c5" in cases:  # 1 MiB, 8192 stripes per GPU (the 64k-stripe / 8-GPU split)
        size, n = 1 << 20, 8192
        t, sh, st = batch(size, n, dev, 4)
        secs = timed(lambda i: x.encode_batched(t.data_ptr(), size, sh, st, n, s), reps=5, warm=1)
        emit("encode", size, n, secs, n * 16 * size, sh)
        secs = timed(lambda i: x.reconst_one_batched(t.data_ptr(), size, sh, st, n, i % D, s),
                     reps=5, warm=1)
        emit("reconst_one", size, n, secs, n * 9 * size, sh)
        del t
    if "multi" in cases:  # Reconst with 2..4 lost data vects (xrs_test.go:530-582)
        for size, n in ((4096, 65536), (1 << 20, 256)):
            t, sh, st = batch(size, n, dev, 5)
            x.encode_batched(t.data_ptr(), size, sh, st, n, s)
            for mode in ("ct", "ct_onewave", "ct_early", "late", "early", "steps"):
                # read per call by the library ("ct": the default, the
                # wave-specialised kernel at 2-3 lost; "ct_onewave": without it)
                os.environ["XRS_RECONST"] = mode
                os.environ["XRS_STAGED_WS"] = "" if mode == "ct" else "0"
                os.environ["XRS_STAGED_LATE"] = "0" if mode == "early" else "1"
                os.environ["XRS_STAGED_CT"] = "1" if mode.startswith("ct") else "0"
                os.environ["XRS_STAGED_EARLY"] = "1" if mode == "ct_early" else "0"
                for lost in (1, 2, 3, 4):
                    need = list(range(lost))
                    has = list(range(lost, D + P))
                    secs = timed(lambda i: x.reconst_batched(t.data_ptr(), size, sh, st, n, has,
                                                             need, s))
                    # xrs_test.go:565-572: one lost data vect is ReconstOne, 9*S
                    per = 9 * size if lost == 1 else (D + lost) * size
                    emit(f"reconst_{lost}_{mode}", size, n, secs, n * per, sh)
            os.environ.pop("XRS_RECONST", None)
            os.environ.pop("XRS_STAGED_LATE", None)
            os.environ.pop("XRS_STAGED_CT", None)
            os.environ.pop("XRS_STAGED_EARLY", None)
            os.environ.pop("XRS_STAGED_WS", None)
            del t
    if "others" in cases:  # other (d, p): runtime-count kernels
        for d, p in ((10, 4), (6, 3), (8, 4), (4, 2), (16, 4), (20, 4), (12, 3)):
            xo = xrs_amd.XRS(d, p)
            for size in (4096, 1 << 20):
                n = (4 << 30) // ((d + p) * size)
                shard, stripe = xrs_amd.batch_strides(size, d + p)
                t = torch.randint(0, 256, (n * stripe,), dtype=torch.uint8, device=dev)
                secs = timed(lambda i: xo.encode_batched(t.data_ptr(), size, shard, stripe, n, s))
                emit(f"encode_{d}+{p}", size, n, secs, n * (d + p) * size, shard)
                a_need, _ = xo.get_need_vects(0)
                secs = timed(lambda i: xo.reconst_one_batched(t.data_ptr(), size, shard, stripe, n,
                                                              0, s))
                emit(f"reconst_one_{d}+{p}", size, n, secs,
                     n * ((d - 1 + 2 + len(a_need)) * size // 2 + size), shard)
                del t
    if "rows_bs" in cases:  # ReconstOne @ 4 KiB: 256- vs 1024-thread blocks, other codecs
        for d, p in ((12, 3), (16, 4), (14, 4), (12, 4), (10, 4)):
            xo = xrs_amd.XRS(d, p)
            size = 4096
            n = (4 << 30) // ((d + p) * size)
            shard, stripe = xrs_amd.batch_strides(size, d + p)
            t = torch.randint(0, 256, (n * stripe,), dtype=torch.uint8, device=dev)
            a_need, _ = xo.get_need_vects(0)
            res = {}
            for rnd in range(2):
                for bs in ("256", "1024"):
                    os.environ["XRS_ROWS_BLOCK"] = bs
                    secs = timed(lambda i: xo.reconst_one_batched(t.data_ptr(), size, shard, stripe,
                                                                  n, 0, s))
                    res[bs] = min(res.get(bs, 1e9), secs)
            os.environ.pop("XRS_ROWS_BLOCK", None)
            for bs, secs in res.items():
                emit(f"reconst_one_{d}+{p}_block_{bs}", size, n, secs,
                     n * ((d - 1 + 2 + len(a_need)) * size // 2 + size), shard)
            del t
    if "replace_ab" in cases:  # Replace(n): compile-time vs runtime source count
        for size, n in ((4096, 65536), (8 << 20, 32)):
            t, sh, st = batch(size, n, dev, 7)
            x.encode_batched(t.data_ptr(), size, sh, st, n, s)
            par = t.data_ptr() + D * sh
            res = {}
            for rnd in range(2):
                for mode in ("ct", "dyn"):
                    if mode == "dyn":
                        os.environ["XRS_REPLACE_DYN"] = "1"
                    else:
                        os.environ.pop("XRS_REPLACE_DYN", None)
                    for nrep in range(1, 9):
                        rows = list(range(nrep))
                        secs = timed(lambda i: x.replace_batched(t.data_ptr(), sh, st, rows, size,
                                                                 par, sh, st, n, s))
                        res[(mode, nrep)] = min(res.get((mode, nrep), 1e9), secs)
            os.environ.pop("XRS_REPLACE_DYN", None)
            for (mode, nrep), secs in sorted(res.items()):
                emit(f"replace_{nrep}_{mode}", size, n, secs, n * (nrep + 2 * P) * size, sh)
            del t
    if "multi_bs" in cases:  # staged Reconst (compile-time kernel) at every block size
        for size, n in ((4096, 65536), (1 << 20, 256)):
            t, sh, st = batch(size, n, dev, 5)
            x.encode_batched(t.data_ptr(), size, sh, st, n, s)
            res = {}
            for rnd in range(2):
                for bs in ("128", "256", "512", "1024"):
                    os.environ["XRS_STAGED_BLOCK"] = bs
                    for lost in (2, 3, 4):
                        need, has = list(range(lost)), list(range(lost, D + P))
                        secs = timed(lambda i: x.reconst_batched(t.data_ptr(), size, sh, st, n,
                                                                 has, need, s))
                        res[(bs, lost)] = min(res.get((bs, lost), 1e9), secs)
            os.environ.pop("XRS_STAGED_BLOCK", None)
            for (bs, lost), secs in sorted(res.items()):
                emit(f"reconst_{lost}_block_{bs}", size, n, secs, n * (D + lost) * size, sh)
            del t
    if "multi_bs_order" in cases:  # staged Reconst: block size x order x early/late
        sizes = ((1 << 20, 256), (256 << 10, 1024), (4096, 65536))
        for size, n in sizes:
            t, sh, st = batch(size, n, dev, 5)
            x.encode_batched(t.data_ptr(), size, sh, st, n, s)
            res = {}
            for rnd in range(2):
                for bs in ("128", "256"):
                    os.environ["XRS_STAGED_BLOCK"] = bs  # (knob removed after this sweep)
                    for early in ("0", "1"):
                        os.environ["XRS_STAGED_EARLY"] = early
                        for order in ("", "0", "16", "32", "64", "128", "256"):
                            if order:
                                os.environ["XRS_BLOCK_ORDER"] = order
                            else:
                                os.environ.pop("XRS_BLOCK_ORDER", None)
                            for lost in (2, 4):
                                need, has = list(range(lost)), list(range(lost, D + P))
                                secs = timed(lambda i: x.reconst_batched(t.data_ptr(), size, sh, st,
                                                                         n, has, need, s), ramp=0.05)
                                k = (bs, early, order or "def", lost)
                                res[k] = min(res.get(k, 1e9), secs)
            for v in ("XRS_STAGED_BLOCK", "XRS_STAGED_EARLY", "XRS_BLOCK_ORDER"):
                os.environ.pop(v, None)
            for (bs, early, order, lost), secs in sorted(res.items()):
                emit(f"reconst_{lost}_bs{bs}_early{early}_order{order}", size, n, secs,
                     n * (D + lost) * size, sh)
            del t
    if "multi_big_bs" in cases:  # staged Reconst, late kernel: 512/1024-thread blocks x order
        for size, n in ((1 << 20, 256), (256 << 10, 1024)):
            t, sh, st = batch(size, n, dev, 5)
            x.encode_batched(t.data_ptr(), size, sh, st, n, s)
            res = {}
            for rnd in range(2):
                for bs in ("", "512", "1024"):
                    if bs:
                        os.environ["XRS_STAGED_BLOCK"] = bs
                    else:
                        os.environ.pop("XRS_STAGED_BLOCK", None)
                    for order in ("", "8", "16", "32", "64", "128"):
                        if order:
                            os.environ["XRS_BLOCK_ORDER"] = order
                        else:
                            os.environ.pop("XRS_BLOCK_ORDER", None)
                        for lost in (2, 4):
                            need, has = list(range(lost)), list(range(lost, D + P))
                            secs = timed(lambda i: x.reconst_batched(t.data_ptr(), size, sh, st, n,
                                                                     has, need, s), ramp=0.05)
                            k = (bs or "def", order or "def", lost)
                            res[k] = min(res.get(k, 1e9), secs)
            for v in ("XRS_STAGED_BLOCK", "XRS_BLOCK_ORDER"):
                os.environ.pop(v, None)
            for (bs, order, lost), secs in sorted(res.items()):
                emit(f"reconst_{lost}_bs{bs}_order{order}", size, n, secs, n * (D + lost) * size, sh)
            del t
    if "multi_big_confirm" in cases:  # staged Reconst: default vs 1024-thread blocks, K 32 / 64
        for size in (512 << 10, 1 << 20, 2 << 20, 8 << 20):
            n = (4 << 30) // (16 * size)
            t, sh, st = batch(size, n, dev, 5)
            x.encode_batched(t.data_ptr(), size, sh, st, n, s)
            res = {}
            for rnd in range(3):
                for bs, order in (("", ""), ("1024", "32"), ("1024", "64"), ("1024", "")):
                    for v, val in (("XRS_STAGED_BLOCK", bs), ("XRS_BLOCK_ORDER", order)):
                        if val:
                            os.environ[v] = val
                        else:
                            os.environ.pop(v, None)
                    for lost in (2, 3, 4):
                        need, has = list(range(lost)), list(range(lost, D + P))
                        secs = timed(lambda i: x.reconst_batched(t.data_ptr(), size, sh, st, n,
                                                                 has, need, s), ramp=0.05)
                        k = (bs or "def", order or "def", lost)
                        res[k] = min(res.get(k, 1e9), secs)
            for v in ("XRS_STAGED_BLOCK", "XRS_BLOCK_ORDER"):
                os.environ.pop(v, None)
            for (bs, order, lost), secs in sorted(res.items()):
                emit(f"reconst_{lost}_bs{bs}_order{order}", size, n, secs, n * (D + lost) * size, sh)
            del t
    if "multi_il" in cases:  # staged Reconst, every load first: a/b of a survivor back to back
        for size, n in ((4096, 65536), (16384, 16384), (64 << 10, 4096), (256 << 10, 1024)):
            t, sh, st = batch(size, n, dev, 5)
            x.encode_batched(t.data_ptr(), size, sh, st, n, s)
            res = {}
            for rnd in range(4):
                for il in ("0", "1"):
                    os.environ["XRS_STAGED_IL"] = il
                    for lost in (2, 3, 4):
                        need, has = list(range(lost)), list(range(lost, D + P))
                        secs = timed(lambda i: x.reconst_batched(t.data_ptr(), size, sh, st, n,
                                                                 has, need, s), ramp=0.05)
                        res[(il, lost)] = min(res.get((il, lost), 1e9), secs)
            os.environ.pop("XRS_STAGED_IL", None)
            for (il, lost), secs in sorted(res.items(), key=lambda kv: (kv[0][1], kv[0][0])):
                emit(f"reconst_{lost}_il{il}", size, n, secs, n * (D + lost) * size, sh)
            del t
    if "multi_mixed" in cases:  # Reconst with lost parity in the loss pattern (xrs.go:236-301)
        # bytes: the reference's accounting generalised, (d + lost) * S per
        # stripe (d survivors read, the lost vects written)
        pats = [([13], [13]), ([12], [12]), ([0, 13], [0, 13]), ([0, 12], [0, 12]),
                ([0, 1, 13], [0, 1, 13]), ([0, 1, 12, 13], [0, 1, 12, 13])]
        for size, n in ((4096, 65536), (1 << 20, 256)):
            t, sh, st = batch(size, n, dev, 5)
            x.encode_batched(t.data_ptr(), size, sh, st, n, s)
            for lost, need in pats:
                has = [i for i in range(D + P) if i not in lost]
                secs = timed(lambda i: x.reconst_batched(t.data_ptr(), size, sh, st, n, has, need, s))
                tag = "lost" + "-".join(map(str, lost)) + "_need" + "-".join(map(str, need))
                emit(f"reconst_{tag}", size, n, secs, n * (D + len(lost)) * size, sh)
            del t
    if "multi_npre" in cases:  # staged Reconst: b-row loads issued with the a-rows
        for size, n in ((4096, 65536), (64 << 10, 4096), (1 << 20, 256)):
            t, sh, st = batch(size, n, dev, 5)
            x.encode_batched(t.data_ptr(), size, sh, st, n, s)
            res = {}
            for rnd in range(3):  # interleaved rounds, best of each
                for npre in ("0", "4", "6", "8", "all"):
                    os.environ["XRS_STAGED_NPRE"] = "-1" if npre == "all" else npre
                    for lost in (2, 3, 4):
                        need, has = list(range(lost)), list(range(lost, D + P))
                        secs = timed(lambda i: x.reconst_batched(t.data_ptr(), size, sh, st, n,
                                                                 has, need, s))
                        res[(npre, lost)] = min(res.get((npre, lost), 1e9), secs)
            os.environ.pop("XRS_STAGED_NPRE", None)
            for (npre, lost), secs in sorted(res.items(), key=lambda kv: (kv[0][1], kv[0][0])):
                emit(f"reconst_{lost}_npre_{npre}", size, n, secs, n * (D + lost) * size, sh)
            del t
    if "multi_order" in cases:  # staged Reconst (compile-time kernel) in every block order
        sizes = ((4096, 65536), (1 << 20, 256))
        if os.environ.get("MULTI_SIZES"):  # e.g. MULTI_SIZES=1048576
            sizes = tuple((int(v), (4 << 30) // (16 * int(v))) for v in
                          os.environ["MULTI_SIZES"].split(","))
        for size, n in sizes:
            t, sh, st = batch(size, n, dev, 5)
            x.encode_batched(t.data_ptr(), size, sh, st, n, s)
            for order in ("", "0", "8", "32", "128", "512", "full"):
                if order:
                    os.environ["XRS_BLOCK_ORDER"] = order
                else:
                    os.environ.pop("XRS_BLOCK_ORDER", None)
                for lost in (2, 3, 4):
                    need, has = list(range(lost)), list(range(lost, D + P))
                    secs = timed(lambda i: x.reconst_batched(t.data_ptr(), size, sh, st, n, has,
                                                             need, s))
                    emit(f"reconst_{lost}_order_{order or 'default'}", size, n, secs,
                         n * (D + lost) * size, sh)
            os.environ.pop("XRS_BLOCK_ORDER", None)
            del t
    if "others_ab" in cases:  # other (d, p): compile-time shapes vs runtime-count kernels
        for d, p in ((10, 4), (6, 3), (8, 4), (4, 2), (16, 4), (20, 4), (12, 3), (14, 4), (10, 2)):
            xo = xrs_amd.XRS(d, p)
            for size in (4096, 1 << 20):
                n = (4 << 30) // ((d + p) * size)
                shard, stripe = xrs_amd.batch_strides(size, d + p)
                t = torch.randint(0, 256, (n * stripe,), dtype=torch.uint8, device=dev)
                ks = sorted({0, d - 1})
                best = {}
                for rnd in range(2):  # interleaved A/B rounds, best of each
                    for mode in ("ct", "dyn"):
                        for var in ("XRS_ENCODE_DYN", "XRS_ROWS_DYN"):
                            if mode == "dyn":
                                os.environ[var] = "1"
                            else:
                                os.environ.pop(var, None)
                        sec = timed(lambda i: xo.encode_batched(t.data_ptr(), size, shard, stripe,
                                                                n, s))
                        best[("enc", mode)] = min(best.get(("enc", mode), 1e9), sec)
                        for k in ks:
                            sec = timed(lambda i: xo.reconst_one_batched(t.data_ptr(), size, shard,
                                                                         stripe, n, k, s))
                            best[(k, mode)] = min(best.get((k, mode), 1e9), sec)
                for var in ("XRS_ENCODE_DYN", "XRS_ROWS_DYN"):
                    os.environ.pop(var, None)
                for mode in ("ct", "dyn"):
                    emit(f"encode_{d}+{p}_{mode}", size, n, best[("enc", mode)],
                         n * (d + p) * size, shard)
                    for k in ks:
                        a_need, _ = xo.get_need_vects(k)
                        emit(f"reconst_one_{d}+{p}_k{k}_{mode}", size, n, best[(k, mode)],
                             n * ((d - 1 + 2 + len(a_need)) * size // 2 + size), shard)
                del t
    torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
