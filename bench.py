#!/usr/bin/env python3
"""Headline benchmark of the MI355X X-Reed-Solomon codec.

Metric (BASELINE.json): "Encode + 1-lost Reconstruct GiB/s (device-resident),
12+4 @ 4KiB/1MiB".  One step = one pass of the hot path over one batch of each
of the four (operation, vect size) pairs the north star names:

  * Encode (xrs.go:103) of `--enc-stripes` 12+4 stripes of 4 KiB vects
    (65,536 stripes = 4 GiB; algorithmic bytes (d+p)*S per stripe, the
    reference's SetBytes, xrs_test.go:513);
  * ReconstOne (xrs.go:175, Reconst with one lost data vect) of the same
    4 KiB stripes (bytes 9*S per stripe = 8*S read + S written,
    xrs_test.go:565-572);
  * Encode of `--rec-stripes` 12+4 stripes of 1 MiB vects (512 stripes = 8 GiB);
  * ReconstOne of the same 1 MiB stripes.

ReconstOne rebuilds data shard k = step mod 12.
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
    """Bytes/s of the oracle's batch path on `threads` for the four bench
    kernels, each run for seconds/4 on a bounded sample."""
    rng = np.random.Generator(np.random.PCG64(1))

    def run(fn, nbytes):
        fn(0)  # warm
        t0, reps = time.perf_counter(), 0
        while True:
            fn(reps)
            reps += 1
            if time.perf_counter() - t0 > seconds / 4:
                break
        return reps * nbytes / (time.perf_counter() - t0)

    rates = {}
    for key, size, n in (("4k", ENC_S, 16384), ("1m", REC_S, 64)):  # 1 GiB each (> LLC)
        buf = rng.integers(0, 256, size=(n, D + P, size), dtype=np.uint8)
        rates["encode_" + key] = run(lambda i: o.encode_batch(buf, size, n, threads),
                                     n * (D + P) * size)
        rates["reconst_one_" + key] = run(
            lambda i: o.reconst_one_batch(buf, size, n, i % D, threads), n * 9 * size)
        del buf
    return rates


def cpu_baseline(seconds: float, step_bytes: dict):
    """The oracle's CPU path (AVX2 low/high-nibble tables + separate piggyback
    pass, i.e. the reference's algorithm) on a bounded sample: 1 thread (the
    reported value), then the box's CPU share (up to 16 threads)."""
    from oracle.oracle_c import OracleXRS, lib

    o = OracleXRS(D, P)

    def mix(rates):  # same byte mix as one GPU step
        t_step = sum(step_bytes[k] / rates[k] for k in step_bytes)
        return sum(step_bytes.values()) / t_step / 2**30

    r1 = _cpu_rates(o, seconds, 1)
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    threads = max(1, min(16, share, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))
    rn = _cpu_rates(o, seconds / 2, threads)
    return {
        "value": round(mix(r1), 3), "unit": "GiB/s", "cores": 1, "kind": "port",
        "simd": ("scalar", "avx2", "avx512bw")[lib().oxrs_simd_level()],
        "cpu_model": _cpu_model(),
        "gibps": {k: round(v / 2**30, 3) for k, v in r1.items()},
        "multi_thread": {"threads": threads, "value": round(mix(rn), 3),
                         "gibps": {k: round(v / 2**30, 3) for k, v in rn.items()}},
        "sample": (f"oracle/xrs_oracle.c: Encode and ReconstOne of 16384 12+4 stripes @ 4 KiB "
                   f"(1 GiB) and of 64 stripes @ 1 MiB (1 GiB), each repeated for "
                   f"{seconds / 4:.1f} s on 1 thread and {seconds / 8:.1f} s on {threads} "
                   f"threads; combined with the GPU step's byte mix"),
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
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--ramp-seconds", type=float, default=0.5)
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
    # shards back to back at 4 KiB and 1 MiB (the kernels' XCD-aware block
    # order makes padding unnecessary below 4 MiB).
    enc_shard, enc_stripe = xrs_amd.batch_strides(ENC_S, D + P)
    rec_shard, rec_stripe = xrs_amd.batch_strides(REC_S, D + P)
    enc_buf = torch.randint(0, 256, (n_enc * enc_stripe,), dtype=torch.uint8, device=dev,
                            generator=g)
    rec_buf = torch.randint(0, 256, (n_rec * rec_stripe,), dtype=torch.uint8, device=dev,
                            generator=g)
    x.encode_batched(enc_buf.data_ptr(), ENC_S, enc_shard, enc_stripe, n_enc, stream)
    x.encode_batched(rec_buf.data_ptr(), REC_S, rec_shard, rec_stripe, n_rec, stream)
    torch.cuda.synchronize()
    # Clock ramp (setup, untimed): an idle MI355X runs its first ~50 launches
    # of this size up to 30% slower (tools/first_alloc_probe.py,
    # profiles/r01_first_alloc.log).  Repeat the (idempotent) setup encode for
    # --ramp-seconds before the W warmup steps.
    t_ramp = time.perf_counter()
    while time.perf_counter() - t_ramp < args.ramp_seconds:
        x.encode_batched(enc_buf.data_ptr(), ENC_S, enc_shard, enc_stripe, n_enc, stream)
        torch.cuda.synchronize()
    # The four timed launches of a step, in order: (key, kernel, algorithmic
    # bytes per launch, read bytes per launch, launcher).
    launches = [
        ("encode_4k", "pair_kernel<4,12,false,true,128>", n_enc * (D + P) * ENC_S, n_enc * D * ENC_S,
         lambda i: x.encode_batched(enc_buf.data_ptr(), ENC_S, enc_shard, enc_stripe, n_enc,
                                    stream)),
        ("reconst_one_4k", "rows_kernel<2,12,4,false,true,256>", n_enc * 9 * ENC_S,
         n_enc * 8 * ENC_S,
         lambda i: x.reconst_one_batched(enc_buf.data_ptr(), ENC_S, enc_shard, enc_stripe, n_enc,
                                         i % D, stream)),
        ("encode_1m", "pair_kernel<4,12,false,true,256>", n_rec * (D + P) * REC_S, n_rec * D * REC_S,
         lambda i: x.encode_batched(rec_buf.data_ptr(), REC_S, rec_shard, rec_stripe, n_rec,
                                    stream)),
        ("reconst_one_1m", "rows_kernel<2,12,4,false,true,1024>", n_rec * 9 * REC_S,
         n_rec * 8 * REC_S,
         lambda i: x.reconst_one_batched(rec_buf.data_ptr(), REC_S, rec_shard, rec_stripe, n_rec,
                                         i % D, stream)),
    ]
    launches = [l for l in launches if l[2] > 0]
    step_bytes = sum(l[2] for l in launches)
    nl = len(launches)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(nl + 1)] for _ in range(args.steps)]

    def step(i, events=None):
        for j, l in enumerate(launches):
            if events:
                events[j].record()
            l[4](i)
        if events:
            events[nl].record()

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
    # Every rank's time (one slot each, summed), so the max and the spread
    # across ranks are both reported.
    t = torch.zeros(world, dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    t[rank] = elapsed
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    rank_seconds = [float(v) for v in t.cpu()]
    elapsed_max = max(rank_seconds)
    total_bytes = world * args.steps * step_bytes
    value = total_bytes / elapsed_max / 2**30

    kernels = {}
    for j, (key, kname, nbytes, rbytes, _) in enumerate(launches):
        ms = float(np.mean([e[j].elapsed_time(e[j + 1]) for e in ev]))
        kernels[key] = {
            "kernel": kname, "ms": round(ms, 4), "bytes_per_launch": nbytes,
            "gibps": round(nbytes / (ms / 1e3) / 2**30, 1),
            "achieved_gbs": round(nbytes / (ms / 1e3) / 1e9, 1),
            "frac": round(nbytes / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "read_only_gbs": round(rbytes / (ms / 1e3) / 1e9, 1),
        }
    dom_key = max(kernels, key=lambda k: kernels[k]["ms"])
    dom = kernels[dom_key]
    traffic = pmc_traffic(dom_key)
    roofline = {
        "bound": "hbm", "kernel": dom["kernel"], "launch": dom_key,
        "achieved": dom["achieved_gbs"],
        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(dom["achieved_gbs"] / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "algorithmic_bytes_per_launch": dom["bytes_per_launch"],
        # the north star's "HBM-read roofline": read bytes only over the same peak
        "read_achieved": dom["read_only_gbs"],
        "read_frac": round(dom["read_only_gbs"] / HBM_PEAK_GBS, 4),
    }

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("timing CPU baseline ...")
        cpu = cpu_baseline(args.cpu_seconds, {l[0]: l[2] for l in launches})

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
                "workload": (f"12+4 Encode + ReconstOne (k = step mod 12) of {n_enc} stripes "
                             f"@ 4 KiB and of {n_rec} stripes @ 1 MiB, per GPU per step"),
                "data_shards": D, "parity_shards": P,
                "encode_vect_bytes": ENC_S, "encode_stripes_per_gpu": n_enc,
                "reconst_vect_bytes": REC_S, "reconst_stripes_per_gpu": n_rec,
                "encode_shard_stride": enc_shard, "reconst_shard_stride": rec_shard,
                "parallelism": f"stripe split x{world}, no collective",
            },
            "rank_seconds": [round(v, 6) for v in rank_seconds],
            "kernels": kernels,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
