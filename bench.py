#!/usr/bin/env python3
"""Headline benchmark of the MI355X X-Reed-Solomon codec.

Metric (BASELINE.json): "Encode + 1-lost Reconstruct GiB/s (device-resident),
12+4 @ 4KiB/1MiB".  One step = one pass of the hot path over one batch:

  * Encode (xrs.go:103) of `--enc-stripes` 12+4 stripes of 4 KiB vects
    (65,536 stripes = 4 GiB; algorithmic bytes (d+p)*S per stripe, the
    reference's SetBytes, xrs_test.go:513), then
  * ReconstOne (xrs.go:175, via Reconst with one lost data vect) of
    `--rec-stripes` 12+4 stripes of 1 MiB vects (512 stripes = 8 GiB buffer;
    bytes 9*S per stripe = 8*S read + S written, xrs_test.go:565-572).

value = algorithmic bytes of all ranks / max-over-ranks time, in GiB/s.  Inputs
are synthetic, generated on the device, and resident in HBM before timing.
Multi-GPU: one process per GPU, each with its own batch (weak scaling, no
collective on the data path; the barrier and the max-time all-reduce only
bracket the timed region).

Prints ONE JSON line on rank 0 (stdout); progress goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import xrs_amd  # noqa: E402

D, P = 12, 4
ENC_S = 4096
REC_S = 1 << 20
HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_rates(o, seconds: float, threads: int):
    """(Encode B/s, ReconstOne B/s) of the oracle's batch path on `threads`."""
    rng = np.random.Generator(np.random.PCG64(1))
    n_enc = 4096  # 256 MiB of 4 KiB stripes
    buf = rng.integers(0, 256, size=(n_enc, D + P, ENC_S), dtype=np.uint8)
    o.encode_batch(buf, ENC_S, n_enc, threads)  # warm
    t0, reps = time.perf_counter(), 0
    while True:
        o.encode_batch(buf, ENC_S, n_enc, threads)
        reps += 1
        if time.perf_counter() - t0 > seconds / 2:
            break
    enc_rate = reps * n_enc * (D + P) * ENC_S / (time.perf_counter() - t0)
    del buf
    n_rec = 64  # 1 GiB of 1 MiB stripes
    buf = rng.integers(0, 256, size=(n_rec, D + P, REC_S), dtype=np.uint8)
    o.encode_batch(buf, REC_S, n_rec, threads)
    t0, reps = time.perf_counter(), 0
    while True:
        o.reconst_one_batch(buf, REC_S, n_rec, reps % D, threads)
        reps += 1
        if time.perf_counter() - t0 > seconds / 2:
            break
    rec_rate = reps * n_rec * 9 * REC_S / (time.perf_counter() - t0)
    return enc_rate, rec_rate


def cpu_baseline(seconds: float, enc_bytes_step: float, rec_bytes_step: float):
    """The oracle's CPU path (AVX2 low/high-nibble tables + separate piggyback
    pass, i.e. the reference's algorithm) on a bounded sample: 1 thread (the
    reported value), then the box's CPU share (up to 16 threads)."""
    from oracle.oracle_c import OracleXRS, lib

    o = OracleXRS(D, P)

    def mix(enc_rate, rec_rate):  # same byte mix as one GPU step
        t_step = enc_bytes_step / enc_rate + rec_bytes_step / rec_rate
        return (enc_bytes_step + rec_bytes_step) / t_step / 2**30

    enc1, rec1 = _cpu_rates(o, seconds, 1)
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    threads = max(1, min(16, share, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))
    encn, recn = _cpu_rates(o, seconds / 2, threads)
    return {
        "value": round(mix(enc1, rec1), 3), "unit": "GiB/s", "cores": 1, "kind": "port",
        "simd": "avx2" if lib().oxrs_simd_available() else "scalar",
        "cpu_model": _cpu_model(),
        "encode_gibps": round(enc1 / 2**30, 3),
        "reconst_one_gibps": round(rec1 / 2**30, 3),
        "multi_thread": {"threads": threads, "value": round(mix(encn, recn), 3),
                         "encode_gibps": round(encn / 2**30, 3),
                         "reconst_one_gibps": round(recn / 2**30, 3)},
        "sample": (f"oracle/xrs_oracle.c: Encode of 4096 12+4 stripes @ 4 KiB (256 MiB) and "
                   f"ReconstOne of 64 stripes @ 1 MiB (1 GiB), repeated for {seconds / 2:.0f} s "
                   f"each on 1 thread and {seconds / 4:.0f} s each on {threads} threads; "
                   f"combined with the GPU step's byte mix"),
    }


def pmc_traffic(kernel_key: str):
    """HBM bytes per launch from profiles/pmc_traffic.json (written by
    tools/pmc_traffic.py from rocprofv3 --pmc passes), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(kernel_key, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--enc-stripes", type=int, default=65536)
    ap.add_argument("--rec-stripes", type=int, default=512)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    # One process per GPU.  XRS_DIST_BACKEND=gloo rehearses N ranks on fewer
    # GPUs (ranks share a card); the driver's runs use nccl (RCCL), one per GPU.
    backend = os.environ.get("XRS_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(local % ndev)
    dev = torch.device("cuda", local % ndev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    def barrier():
        if world > 1:
            dist.barrier()

    x = xrs_amd.XRS(D, P)
    stream = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED + rank)
    n_enc, n_rec = args.enc_stripes, args.rec_stripes
    # Device batch layout: the library's recommended strides (xrs_batch_strides):
    # 4 KiB vects back to back, 1 MiB vects with a 256 B pad per shard.
    enc_shard, enc_stripe = xrs_amd.batch_strides(ENC_S, D + P)
    rec_shard, rec_stripe = xrs_amd.batch_strides(REC_S, D + P)
    enc_buf = torch.randint(0, 256, (n_enc * enc_stripe,), dtype=torch.uint8, device=dev,
                            generator=g)
    rec_buf = torch.randint(0, 256, (n_rec * rec_stripe,), dtype=torch.uint8, device=dev,
                            generator=g)
    x.encode_batched(rec_buf.data_ptr(), REC_S, rec_shard, rec_stripe, n_rec, stream)
    torch.cuda.synchronize()
    enc_bytes = n_enc * (D + P) * ENC_S          # per launch, algorithmic (read + write)
    rec_bytes = n_rec * 9 * REC_S

    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]

    def step(i, events=None):
        if events:
            events[0].record()
        if n_enc:
            x.encode_batched(enc_buf.data_ptr(), ENC_S, enc_shard, enc_stripe, n_enc, stream)
        if events:
            events[1].record()
        if n_rec:
            x.reconst_one_batched(rec_buf.data_ptr(), REC_S, rec_shard, rec_stripe, n_rec,
                                  i % D, stream)
        if events:
            events[2].record()

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, ev[i])
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    barrier()
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed_max = float(t.item())

    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    rec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))
    total_bytes = world * args.steps * (enc_bytes + rec_bytes)
    value = total_bytes / elapsed_max / 2**30

    kernels = {}
    if n_enc:
        kernels["encode_4k"] = {
            "kernel": "pair_kernel<4,12,false,true>", "ms": round(enc_ms, 4),
            "bytes_per_launch": enc_bytes,
            "gibps": round(enc_bytes / (enc_ms / 1e3) / 2**30, 1),
            "achieved_gbs": round(enc_bytes / (enc_ms / 1e3) / 1e9, 1),
            "read_only_gbs": round(n_enc * D * ENC_S / (enc_ms / 1e3) / 1e9, 1),
        }
    if n_rec:
        kernels["reconst_one_1m"] = {
            "kernel": "rows_kernel<2,12,4,false,true>", "ms": round(rec_ms, 4),
            "bytes_per_launch": rec_bytes,
            "gibps": round(rec_bytes / (rec_ms / 1e3) / 2**30, 1),
            "achieved_gbs": round(rec_bytes / (rec_ms / 1e3) / 1e9, 1),
            "read_only_gbs": round(n_rec * 8 * REC_S / (rec_ms / 1e3) / 1e9, 1),
        }
    dom_key = max(kernels, key=lambda k: kernels[k]["ms"])
    dom = kernels[dom_key]
    traffic = pmc_traffic(dom_key)
    roofline = {
        "bound": "hbm", "kernel": dom["kernel"], "achieved": dom["achieved_gbs"],
        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(dom["achieved_gbs"] / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "algorithmic_bytes_per_launch": dom["bytes_per_launch"],
    }

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("timing CPU baseline ...")
        cpu = cpu_baseline(args.cpu_seconds, enc_bytes, rec_bytes)

    if rank == 0:
        out = {
            "metric": "Encode + 1-lost Reconstruct GiB/s (device-resident), 12+4 @ 4KiB/1MiB",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (uniform random bytes generated on device, seeded per rank)",
            "config": {
                "workload": (f"12+4 Encode of {n_enc} stripes @ 4 KiB + ReconstOne (k = step mod 12)"
                             f" of {n_rec} stripes @ 1 MiB per GPU per step"),
                "data_shards": D, "parity_shards": P,
                "encode_vect_bytes": ENC_S, "encode_stripes_per_gpu": n_enc,
                "reconst_vect_bytes": REC_S, "reconst_stripes_per_gpu": n_rec,
                "encode_shard_stride": enc_shard, "reconst_shard_stride": rec_shard,
                "parallelism": f"stripe split x{world}, no collective",
            },
            "kernels": kernels,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
