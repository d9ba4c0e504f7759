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

Multi-GPU (xrs_amd/dist.py): one process per GPU.  Under torchrun the ranks
come from WORLD_SIZE (which must equal --gpus); `python bench.py --gpus N`
without a launcher starts the N rank processes itself before any GPU call.
Each rank owns its own batch (weak scaling, no collective on the data path;
the barrier and the per-rank time gather only bracket the timed regions, over
gloo by default: no shard byte crosses ranks, so RCCL has nothing to carry).

After the headline timed region, the same line carries:
  * "config5": BASELINE config 5, Encode + ReconstOne of --config5-stripes
    stripes of 1 MiB vects per rank (8,192 = 128 GiB resident per GPU; at
    N = 8 the 65,536-stripe, 1 TiB batch split 8 ways), with its own
    per-rank times;
  * "config4": BASELINE config 4, Update and Replace(4) of 8 MiB stripes,
    device-resident, with oracle-checked samples;
  * "host_e2e": the host-resident path (shards start and end in pinned host
    memory, xrs_*_host, PCIe-inclusive) on every rank at once;
  * "per_stripe_queue" (N = 1): the reference's per-stripe Encode call from
    32 caller threads through the batching queue, and ("plain_api") the plain
    xrs_encode / xrs_update per stripe from 32 threads on one codec
    (tools/sync_bench children, host-resident 4 KiB stripes, PCIe-inclusive);
  * "xgmi_repair" (two or more visible GPUs): rank 0 (in a child process)
    rebuilds a data shard with half of its need set on the peer GPU (xGMI
    reads), checked bit for bit against the rebuild from local shards.
  * "parity": after the timed regions, each headline launch runs once more
    over a batch whose first / middle / last stripes were poisoned (parity
    for Encode, shard k in {0, 7} for ReconstOne); the checker leg compares
    those stripes with the C oracle (oracle/xrs_oracle.c), on every rank;
  * "rank_devices": every rank's device index and PCI address.  Two ranks on
    one GPU stop the run (exit 3) unless XRS_REHEARSAL=1, which labels the
    line "shared_gpu": true.

Prints ONE JSON line on rank 0 (stdout); progress goes to stderr.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _load_dist():
    """xrs_amd/dist.py without the package __init__ (which loads the HIP
    library): the parent of a self-launched run must not touch the GPU."""
    spec = importlib.util.spec_from_file_location("xrs_bench_dist",
                                                  os.path.join(ROOT, "xrs_amd", "dist.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = mod
    spec.loader.exec_module(mod)
    return mod


xdist = _load_dist()

D, P = 12, 4
ENC_S = 4096
REC_S = 1 << 20
C4_S = 8 << 20  # BASELINE config 4: Update + Replace(4) @ 8 MiB
C4_STRIPES = 16  # CPU sample per op
C4_ROWS = (0, 1, 2, 3)
HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md
GIB = float(1 << 30)


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


def _cpu_samples():
    """The CPU baseline's bounded sample, made once: 12+4 stripes of 4 KiB
    (16,384 = 1 GiB) and 1 MiB (64 = 1 GiB); config 4: 16 stripes of [old,
    new, 4 parity] (768 MiB) and of [4 data, 4 parity] (1 GiB) @ 8 MiB."""
    import numpy as np

    rng = np.random.Generator(np.random.PCG64(1))
    return {
        "4k": rng.integers(0, 256, size=(16384, D + P, ENC_S), dtype=np.uint8),
        "1m": rng.integers(0, 256, size=(64, D + P, REC_S), dtype=np.uint8),
        "upd": rng.integers(0, 256, size=(C4_STRIPES, 2 + P, C4_S), dtype=np.uint8),
        "rep": rng.integers(0, 256, size=(C4_STRIPES, len(C4_ROWS) + P, C4_S), dtype=np.uint8),
    }


def _cpu_rates(o, seconds: float, threads: int, bufs: dict):
    """Bytes/s of the oracle's batch path on `threads` for the four bench
    kernels and BASELINE config 4 (Update, Replace(4) @ 8 MiB), each run for
    seconds/6 on the bounded sample `bufs` (_cpu_samples)."""

    def run(fn, nbytes):
        fn(0)  # warm
        t0, reps = time.perf_counter(), 0
        while True:
            fn(reps)
            reps += 1
            if time.perf_counter() - t0 > seconds / 6:
                break
        return reps * nbytes / (time.perf_counter() - t0)

    rates = {}
    for key, size in (("4k", ENC_S), ("1m", REC_S)):
        buf = bufs[key]
        n = buf.shape[0]
        rates["encode_" + key] = run(lambda i: o.encode_batch(buf, size, n, threads),
                                     n * (D + P) * size)
        rates["reconst_one_" + key] = run(
            lambda i: o.reconst_one_batch(buf, size, n, i % D, threads), n * 9 * size)
    # config 4: bytes (2p+2)*S and (n+2p)*S per stripe (xrs_test.go:600-680)
    rates["update_8m"] = run(lambda i: o.update_batch(bufs["upd"], C4_S, C4_STRIPES, i % D, threads),
                             C4_STRIPES * (2 * P + 2) * C4_S)
    rates["replace4_8m"] = run(
        lambda i: o.replace_batch(bufs["rep"], C4_S, C4_STRIPES, C4_ROWS, threads),
        C4_STRIPES * (len(C4_ROWS) + 2 * P) * C4_S)
    return rates


def _cpu_counts() -> dict:
    """nproc, the affinity set and the cgroup CPU quota (cpu.max) of this
    process: the host's cores and the share of them this job may use."""
    out = {"nproc": os.cpu_count() or 1}
    try:
        out["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        out["affinity"] = out["nproc"]
    out["cgroup_quota_cpus"] = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            out["cgroup_quota_cpus"] = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return out


def cpu_baseline(seconds: float, step_bytes: dict):
    """The oracle's CPU path (AVX2/AVX-512 low/high-nibble tables + separate
    piggyback pass, i.e. the reference's algorithm) on a bounded sample: 1
    thread (the reported value), then every CPU in this process's affinity set
    (uncapped), and the cgroup quota's CPU count when that is smaller."""
    from oracle.oracle_c import OracleXRS, lib

    o = OracleXRS(D, P)

    def mix(rates):  # same byte mix as one GPU step
        t_step = sum(step_bytes[k] / rates[k] for k in step_bytes)
        return sum(step_bytes.values()) / t_step / GIB

    counts = _cpu_counts()
    bufs = _cpu_samples()
    r1 = _cpu_rates(o, seconds, 1, bufs)
    tcounts = [counts["affinity"]]
    q = counts["cgroup_quota_cpus"]
    if q and int(q) >= 1 and int(q) < counts["affinity"]:
        tcounts.append(int(q))
    multi = []
    for t in tcounts:
        rn = _cpu_rates(o, seconds / 2, t, bufs)
        multi.append({"threads": t, "value": round(mix(rn), 3),
                      "gibps": {k: round(v / GIB, 3) for k, v in rn.items()}})
    best = max(multi, key=lambda m: m["value"])
    return {
        "value": round(mix(r1), 3), "unit": "GiB/s", "cores": 1, "kind": "port",
        "simd": ("scalar", "avx2", "avx512bw")[lib().oxrs_simd_level()],
        "cpu_model": _cpu_model(), "cpu_counts": counts,
        "gibps": {k: round(v / GIB, 3) for k, v in r1.items()},
        "multi_thread": best, "multi_thread_all": multi,
        "sample": (f"oracle/xrs_oracle.c: Encode and ReconstOne of 16384 12+4 stripes @ 4 KiB "
                   f"(1 GiB) and of 64 stripes @ 1 MiB (1 GiB); Update and Replace(rows "
                   f"{list(C4_ROWS)}) of {C4_STRIPES} stripes @ 8 MiB (config 4); each repeated "
                   f"for {seconds / 6:.1f} s on 1 thread and {seconds / 12:.1f} s on each of "
                   f"{tcounts} threads; value combines the four headline kernels with the GPU "
                   f"step's byte mix"),
    }


def lib_sha256(path: str) -> str:
    import hashlib

    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def library_info(xa) -> dict:
    """The measured binary and the tree it came from: xrs_version() carries the
    digest of the sources the library was built from (xrs_amd/csrc/version.cpp),
    recomputed here from this checkout."""
    built, tree = xa.library_source_hash(), xa.source_hash()
    return {"path": os.path.relpath(xa.LIB_PATH, ROOT), "version": xa.version(),
            "sha256": lib_sha256(xa.LIB_PATH), "src_hash": built, "tree_src_hash": tree,
            "built_from_tree": built == tree}


def pmc_traffic(launch: str, kernel: str, lib_path: str):
    """(HBM bytes per launch, provenance) from profiles/pmc_traffic.json
    (tools/pmc_traffic.py over two rocprofv3 --pmc passes of this bench).  An
    entry counts only when it names this launch, this kernel and the sha256
    of the library this process loaded: after any rebuild the stored counters
    describe other code, and the line reports traffic null."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            ent = json.load(f).get(launch)
        sha = lib_sha256(lib_path)
    except (OSError, ValueError):
        return None, "profiles/pmc_traffic.json unreadable"
    if not isinstance(ent, dict):
        return None, f"no PMC entry for {launch}"
    if ent.get("kernel") != kernel:
        return None, f"PMC entry is for kernel {ent.get('kernel')!r}, not {kernel!r}"
    if ent.get("lib_sha256") != sha:
        return None, (f"PMC entry measured library sha256 {str(ent.get('lib_sha256'))[:12]}, "
                      f"loaded library is {sha[:12]}")
    return ent.get("hbm_bytes_per_launch"), (
        f"profiles/pmc_traffic.json[{launch}]: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over "
        f"this bench, library sha256 {sha[:12]} (the loaded one)")


# ---------------------------------------------------------------- parity leg
# Driver-visible bit-exactness: after the timed regions, each headline launch
# runs once more (full grid, same kernel shape) over a batch whose sample
# stripes were poisoned first; the sample stripes' bytes before and after come
# back to the host, and the checker leg (with cpu_baseline, never timed)
# compares them with the C oracle.  Reference semantics: Encode xrs.go:103-128,
# ReconstOne xrs.go:175-221.
PARITY_K = (0, 7)


def parity_capture(R: "Rank", tag: str, buf, size: int, shard: int, stripe: int, n: int):
    """GPU half of the parity leg for one vect size: returns [(key, op, k,
    stripes, before, got)], `before` the oracle's input and `got` the GPU's
    output for the sample stripes ([len(stripes), D+P, size] uint8)."""
    torch, x, s = R.torch, R.x, R.stream
    idx = sorted({0, n // 2, n - 1})
    view = buf.view(n, stripe)

    def grab():
        return torch.stack([torch.stack([view[t, i * shard:i * shard + size] for i in range(D + P)])
                            for t in idx]).cpu().numpy()

    out = []
    for t in idx:  # Encode: parity of the samples poisoned, then a full launch
        for i in range(D, D + P):
            view[t, i * shard:i * shard + size].fill_(0xA5)
    R.sync()
    before = grab()
    x.encode_batched(buf.data_ptr(), size, shard, stripe, n, s)
    R.sync()
    out.append(("encode_" + tag, "encode", -1, idx, before, grab()))
    for k in PARITY_K:  # ReconstOne k: shard k of the samples poisoned
        for t in idx:
            view[t, k * shard:k * shard + size].fill_(0x5A)
        R.sync()
        before = grab()
        x.reconst_one_batched(buf.data_ptr(), size, shard, stripe, n, k, s)
        R.sync()
        out.append(("reconst_one_" + tag, "reconst_one", k, idx, before, grab()))
    return out


def oracle_parity(samples):
    """Checker half of the parity leg: the C oracle (oracle/xrs_oracle.c) on
    each sample's `before`, compared byte for byte with the GPU's output."""
    import numpy as np

    from oracle.oracle_c import OracleXRS

    o = OracleXRS(D, P)
    res = {"oracle": "oracle/xrs_oracle.c", "cases": []}
    for key, op, k, idx, before, got in samples:
        ref = before.copy()
        for j in range(ref.shape[0]):
            if op == "update":  # [old, new, parity]
                o.update(ref[j, 0], ref[j, 1], k, [ref[j, 2 + r] for r in range(P)])
                continue
            if op == "replace4":  # [data 0..3, parity]
                nr = len(C4_ROWS)
                o.replace([ref[j, i] for i in range(nr)], list(C4_ROWS),
                          [ref[j, nr + r] for r in range(P)])
                continue
            vects = [ref[j, i] for i in range(D + P)]
            if op == "encode":
                o.encode(vects)
            else:
                o.reconst_one(vects, k)
        ok = bool(np.array_equal(ref, got))
        res[key] = res.get(key, True) and ok
        res["cases"].append({"launch": key, "k": None if k < 0 else k, "stripes": idx,
                             "vect_bytes": int(before.shape[2]), "bitexact": ok})
    return res


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default: WORLD_SIZE, else 1")
    # 1,500 steps = ~4.9 s of timed GPU work at N = 1, so the driver's
    # GPU-busy sampling can see it (1,000 steps read within 0.2% of 200:
    # profiles/r02_steps_ab.jsonl); the whole run stays under a minute
    ap.add_argument("--steps", type=int, default=1500)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--enc-stripes", type=int, default=65536)
    ap.add_argument("--rec-stripes", type=int, default=512)
    ap.add_argument("--config5-stripes", type=int, default=8192,
                    help="1 MiB stripes per rank for the config5 key (0: skip)")
    ap.add_argument("--config5-steps", type=int, default=20)  # ~3.5 s of GPU work
    ap.add_argument("--config4-stripes", type=int, default=64,
                    help="8 MiB stripes per op for the config4 key (0: skip)")
    ap.add_argument("--config4-steps", type=int, default=10)
    ap.add_argument("--host-mib", type=int, default=1024,
                    help="MiB per host-resident batch for the host_e2e key (0: skip)")
    ap.add_argument("--queue-callers", type=int, nargs="*", default=[32],
                    help="caller threads for the per_stripe_queue key (N = 1 only; none: skip)")
    ap.add_argument("--async-window", type=int, default=16,
                    help="stripes each caller keeps in flight in the per_stripe_queue async leg")
    ap.add_argument("--async-callers", type=int, nargs="*", default=[4, 16],
                    help="caller threads of the per_stripe_queue async leg")
    ap.add_argument("--xgmi-stripes", type=int, default=64,
                    help="1 MiB stripes for the xgmi_repair key (0: skip)")
    ap.add_argument("--xgmi-child", type=int, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    # Untimed soak of the headline Encode before the warmup: clock ramp, and
    # >= 6 s of GPU work so a sampler polling GPU busy every few seconds sees
    # the run whatever --steps is.
    ap.add_argument("--ramp-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the post-timing oracle parity leg")
    return ap.parse_args(argv)


class Rank:
    """Per-rank state: device, stream, codec and the timing bracket."""

    def __init__(self, w, backend: str):
        import torch

        import xrs_amd

        self.torch, self.xrs_amd, self.w = torch, xrs_amd, w
        self.ndev = torch.cuda.device_count()
        if self.ndev < 1:
            raise RuntimeError("bench.py needs a GPU (there is no CPU fallback)")
        self.rehearsal = xdist.rehearsal_env()
        # local rank -> visible device; with fewer devices than ranks the PCI
        # check below refuses the run unless it is a labelled rehearsal (a
        # launcher that gives each rank its own single visible GPU passes it)
        self.dev_index = w.local % self.ndev
        torch.cuda.set_device(self.dev_index)
        self.dev = torch.device("cuda", self.dev_index)
        xdist.init(w, backend, self.dev)
        pr = torch.cuda.get_device_properties(self.dev_index)
        me = {"rank": w.rank, "device": self.dev_index,
              "pci": f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}",
              "uuid": str(getattr(pr, "uuid", ""))}
        # every rank's device, checked distinct by PCI address (XRS_REHEARSAL=1
        # allows sharing and labels the line)
        self.rank_devices = xdist.gather_objects(me)
        self.shared_gpu = xdist.check_distinct_devices(self.rank_devices, self.rehearsal)
        # the time gather runs on the device for RCCL, on the host for gloo
        self.tdev = self.dev if (w.world > 1 and backend == "nccl") else None
        self.x = xrs_amd.XRS(D, P)
        self.stream = torch.cuda.current_stream().cuda_stream

    def sync(self):
        self.torch.cuda.synchronize()

    def timed(self, step, steps, warmup):
        return xdist.timed_steps(step, steps, warmup, self.sync, self.tdev)

    def random_bytes(self, n: int, seed: int):
        """n uniform random bytes on the device, filled 1 GiB at a time."""
        torch = self.torch
        buf = torch.empty(n, dtype=torch.uint8, device=self.dev)
        g = torch.Generator(device=self.dev)
        g.manual_seed(seed)
        step = 1 << 30
        for a in range(0, n, step):
            buf[a:a + step].random_(0, 256, generator=g)
        return buf

    def ramp(self, fn, seconds: float):
        """Clock ramp (untimed): an idle MI355X runs its first ~50 launches of
        this size up to 30% slower (tools/first_alloc_probe.py,
        profiles/r01_first_alloc.log)."""
        t = time.perf_counter()
        while time.perf_counter() - t < seconds:
            fn()
            self.sync()


def headline(R: Rank, args):
    """The metric's timed region: the four launches of one step."""
    torch, x, s = R.torch, R.x, R.stream
    n_enc, n_rec = args.enc_stripes, args.rec_stripes
    # Device batch layout: the library's recommended strides (xrs_batch_strides):
    # shards back to back at 4 KiB and 1 MiB (the kernels' XCD-aware block
    # order makes padding unnecessary below 4 MiB).
    enc_shard, enc_stripe = R.xrs_amd.batch_strides(ENC_S, D + P)
    rec_shard, rec_stripe = R.xrs_amd.batch_strides(REC_S, D + P)
    first_enc = xdist.stripe_range(n_enc * R.w.world, R.w.rank, R.w.world)[0]
    enc_buf = R.random_bytes(n_enc * enc_stripe, 0x5EED + first_enc)
    rec_buf = R.random_bytes(n_rec * rec_stripe, 0xB1D + first_enc)
    x.encode_batched(enc_buf.data_ptr(), ENC_S, enc_shard, enc_stripe, n_enc, s)
    x.encode_batched(rec_buf.data_ptr(), REC_S, rec_shard, rec_stripe, n_rec, s)
    R.sync()
    R.ramp(lambda: x.encode_batched(enc_buf.data_ptr(), ENC_S, enc_shard, enc_stripe, n_enc, s),
           args.ramp_seconds)
    # The four timed launches of a step, in order: (key, expected kernel,
    # algorithmic bytes per launch, read bytes per launch, launcher).  The
    # line reports the kernel the library actually launched (traced below).
    launches = [
        ("encode_4k", "enc_ws_kernel<12, 256>", n_enc * (D + P) * ENC_S, n_enc * D * ENC_S,
         lambda i: x.encode_batched(enc_buf.data_ptr(), ENC_S, enc_shard, enc_stripe, n_enc, s)),
        ("reconst_one_4k", "rows_kernel<2, 12, 4, false, true, 256>", n_enc * 9 * ENC_S,
         n_enc * 8 * ENC_S,
         lambda i: x.reconst_one_batched(enc_buf.data_ptr(), ENC_S, enc_shard, enc_stripe, n_enc,
                                         i % D, s)),
        ("encode_1m", "pair_kernel<4, 12, false, true, 128, true>", n_rec * (D + P) * REC_S, n_rec * D * REC_S,
         lambda i: x.encode_batched(rec_buf.data_ptr(), REC_S, rec_shard, rec_stripe, n_rec, s)),
        ("reconst_one_1m", "rows_kernel<2, 12, 4, false, true, 1024>", n_rec * 9 * REC_S,
         n_rec * 8 * REC_S,
         lambda i: x.reconst_one_batched(rec_buf.data_ptr(), REC_S, rec_shard, rec_stripe, n_rec,
                                         i % D, s)),
    ]
    launches = [l for l in launches if l[2] > 0]
    step_bytes = sum(l[2] for l in launches)
    nl = len(launches)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(nl + 1)] for _ in range(args.steps)]
    state = {"timed": False, "i": 0}

    def step(i):
        events = ev[state["i"]] if state["timed"] else None
        for j, l in enumerate(launches):
            if events:
                events[j].record()
            l[4](i)
        if events:
            events[nl].record()
            state["i"] += 1

    # The kernel each launch runs, read from the library's launch trace
    # (one untimed call each): the names rocprofv3 reports.
    traced = {}
    for key, _, _, _, fn in launches:
        R.xrs_amd.trace_kernels(True)
        fn(0)
        R.xrs_amd.trace_kernels(False)
        traced[key] = "; ".join(R.xrs_amd.traced_kernels()) or "?"
    # warmup steps untimed, then exactly args.steps timed ones (with events)
    for i in range(args.warmup):
        step(i)
    state["timed"] = True
    rank_seconds = R.timed(step, args.steps, 0)

    kernels = {}
    for j, (key, _, nbytes, rbytes, _) in enumerate(launches):
        ms = sum(e[j].elapsed_time(e[j + 1]) for e in ev) / len(ev)
        kernels[key] = {
            "kernel": traced[key], "ms": round(ms, 4), "bytes_per_launch": nbytes,
            "gibps": round(nbytes / (ms / 1e3) / GIB, 1),
            "achieved_gbs": round(nbytes / (ms / 1e3) / 1e9, 1),
            "frac": round(nbytes / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "read_only_gbs": round(rbytes / (ms / 1e3) / 1e9, 1),
            "read_frac": round(rbytes / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
        }
    samples = []
    if not args.no_parity:  # untimed: the timed region has ended on every rank
        if n_enc > 0:
            samples += parity_capture(R, "4k", enc_buf, ENC_S, enc_shard, enc_stripe, n_enc)
        if n_rec > 0:
            samples += parity_capture(R, "1m", rec_buf, REC_S, rec_shard, rec_stripe, n_rec)
    del enc_buf, rec_buf
    torch.cuda.empty_cache()
    return launches, step_bytes, rank_seconds, kernels, (enc_shard, rec_shard), samples


def config5_plan(requested: int, fits: int, rank: int, world: int, gather=None) -> dict:
    """Config 5's split (no GPU call): every rank runs the same count -- the
    requested one per rank, or what the emptiest GPU's free HBM holds, agreed
    over the ranks by `gather` (xdist.gather_seconds: one value per rank) --
    and rank r takes the contiguous range xdist.stripe_range(total, r, world).
    At 8 ranks and 8,192 requested: 65,536 stripes, 8,192 per GPU."""
    mine = float(min(requested, fits))
    per_rank = int(min(gather(mine) if gather else [mine]))
    total = per_rank * world
    first, n = xdist.stripe_range(total, rank, world) if per_rank > 0 else (0, 0)
    return {"per_rank": per_rank, "total": total, "first": first, "n": n}


def config5(R: Rank, args):
    """BASELINE config 5: Encode and ReconstOne of 1 MiB stripes, a fixed
    number per rank (8,192 = 128 GiB per GPU; 65,536 stripes = 1 TiB over 8),
    split by xdist.stripe_range; no collective.  Reference workload:
    xrs_test.go:476-480 (1 MiB Encode), xrs.go:175-221 (ReconstOne)."""
    torch, x, s = R.torch, R.x, R.stream
    w = R.w
    shard, stripe = R.xrs_amd.batch_strides(REC_S, D + P)
    # Every rank runs the same count: the requested one, or what the
    # emptiest GPU's free HBM holds (minus 4 GiB), agreed over the ranks.
    free, _ = torch.cuda.mem_get_info()
    fits = max(0, (free - (4 << 30)) // stripe)
    plan = config5_plan(args.config5_stripes, fits, w.rank, w.world,
                        lambda v: xdist.gather_seconds(v, R.tdev))
    if plan["per_rank"] < 1:
        return {"skipped": f"no room for one 16 MiB stripe ({free / GIB:.1f} GiB free)"}
    total, first, n = plan["total"], plan["first"], plan["n"]
    t0 = time.perf_counter()
    buf = R.random_bytes(n * stripe, 0xC05 + first)
    base = buf.data_ptr()
    x.encode_batched(base, REC_S, shard, stripe, n, s)
    R.sync()
    log(f"rank {w.rank}: config5 batch of {n} stripes ({n * stripe / GIB:.1f} GiB) ready in "
        f"{time.perf_counter() - t0:.1f} s")
    R.ramp(lambda: x.encode_batched(base, REC_S, shard, stripe, n, s), 0.2)
    enc_sec = R.timed(lambda i: x.encode_batched(base, REC_S, shard, stripe, n, s),
                      args.config5_steps, 1)
    rec_sec = R.timed(lambda i: x.reconst_one_batched(base, REC_S, shard, stripe, n, i % D, s),
                      args.config5_steps, 1)
    # Round trip on a sample (no oracle on the product path): erase shard k of
    # the first stripes, rebuild the whole batch, compare with the saved bytes.
    k, m = 7, min(n, 64)
    view = buf.view(n, stripe)[:m, k * shard:k * shard + REC_S]
    saved = view.clone()
    view.zero_()
    x.reconst_one_batched(base, REC_S, shard, stripe, n, k, s)
    R.sync()
    ok = bool(torch.equal(view, saved))
    oks = [v > 0.5 for v in xdist.gather_seconds(1.0 if ok else 0.0, R.tdev)]  # every rank's check
    del buf, view, saved
    torch.cuda.empty_cache()
    enc_bytes, rec_bytes = n * (D + P) * REC_S, n * 9 * REC_S
    steps = args.config5_steps
    enc_t, rec_t = max(enc_sec), max(rec_sec)
    world_bytes = lambda per: per * w.world  # every rank holds the same count (+-1 stripe)
    return {
        "workload": (f"12+4 @ 1 MiB: {total} stripes ({total * (D + P) * REC_S / 2**40:.3f} TiB) "
                     f"split {n} per GPU over {w.world} GPU(s), no collective"),
        "stripes_total": total, "stripes_per_rank": n, "stripes_requested": args.config5_stripes,
        "steps": steps,
        "encode": {"rank_seconds": [round(v, 6) for v in enc_sec],
                   "gibps": round(world_bytes(enc_bytes) * steps / enc_t / GIB, 1),
                   "frac_per_gpu": round(enc_bytes * steps / enc_t / 1e9 / HBM_PEAK_GBS, 4)},
        "reconst_one": {"rank_seconds": [round(v, 6) for v in rec_sec],
                        "gibps": round(world_bytes(rec_bytes) * steps / rec_t / GIB, 1),
                        "frac_per_gpu": round(rec_bytes * steps / rec_t / 1e9 / HBM_PEAK_GBS, 4)},
        "gibps": round(world_bytes(enc_bytes + rec_bytes) * steps / (enc_t + rec_t) / GIB, 1),
        "roundtrip_ok": all(oks), "roundtrip_ok_ranks": oks,
    }


def config4(R: Rank, args):
    """BASELINE config 4: Update (row = step mod 12) and Replace(rows 0..3) of
    12+4 stripes of 8 MiB vects, device-resident, batched (xrs_update_batched /
    xrs_replace_batched).  Stripe layouts: [old, new, parity 0..3] and
    [data 0..3, parity 0..3].  Bytes per stripe are the reference's SetBytes
    (xrs_test.go:600-680): (2p+2)*S for Update, (n+2p)*S for Replace(n).
    Each op's first / last stripes are checked against the C oracle in the
    checker leg (samples)."""
    torch, x, s = R.torch, R.x, R.stream
    S, n_upd, n_rep, nr = C4_S, args.config4_stripes, args.config4_stripes, len(C4_ROWS)
    out, samples = {"vect_bytes": S, "replace_rows": list(C4_ROWS)}, []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn, reps):
        fn(0)
        R.sync()
        e0.record()
        for i in range(reps):
            fn(i)
        e1.record()
        R.sync()
        return e0.elapsed_time(e1) / reps / 1e3

    for op, rows_per, n in (("update", 2 + P, n_upd), ("replace4", nr + P, n_rep)):
        # the library's recommended layout for rows_per vects of 8 MiB per
        # stripe (xrs_batch_strides: a 4 KiB + 256 B pad per vect from 4 MiB)
        sh, stripe = R.xrs_amd.batch_strides(S, rows_per)
        buf = R.random_bytes(n * stripe, 0xC04 + len(op))
        b = buf.data_ptr()
        par = (2 if op == "update" else nr) * sh  # parity offset in a stripe
        if op == "update":
            fn = lambda i: x.update_batched(b, stripe, b + sh, stripe, S, i % D, b + par, sh, stripe, n, s)
            algo = n * (2 * P + 2) * S
        else:
            fn = lambda i: x.replace_batched(b, sh, stripe, list(C4_ROWS), S, b + par, sh, stripe, n, s)
            algo = n * (nr + 2 * P) * S
        sec = timed(fn, args.config4_steps)
        idx = [0, n - 1]
        view = buf.view(n, stripe)
        R.sync()

        def grab():
            return torch.stack([torch.stack([view[t, i * sh:i * sh + S] for i in range(rows_per)])
                                for t in idx]).cpu().numpy()

        before = grab()
        row = 5
        if op == "update":
            x.update_batched(b, stripe, b + sh, stripe, S, row, b + par, sh, stripe, n, s)
        else:
            fn(0)
        R.sync()
        got = grab()
        samples.append(("config4_" + op, op, row if op == "update" else -1, idx, before, got))
        out[op] = {"stripes": n, "bytes_per_launch": algo, "ms": round(sec * 1e3, 4),
                   "shard_stride": sh, "stripe_stride": stripe,
                   "gibps": round(algo / sec / GIB, 1), "frac": round(algo / sec / 1e9 / HBM_PEAK_GBS, 4)}
        del buf, view
        torch.cuda.empty_cache()
    return out, samples


def host_e2e(R: Rank, args):
    """Shards start and end in host memory: pinned, device-mapped batches
    (xrs_host_alloc) run by xrs_encode_host / xrs_reconst_one_host, every rank
    at once over its own link, two ways:
      * top-level keys: in place over PCIe (the kernels read and write the
        pinned batch through its device address; the default);
      * "dma": the north star's "pinned hipMemcpyAsync in and out" -- the same
        batches with XRS_HOST_ZC=0, i.e. 64 MiB chunks through three device
        slots and streams, H2D / kernel / D2H overlapped (codec.cpp
        run_pipeline); ReconstOne moves only its need set.
    Reference call sites: xrs.go:103-128 (Encode), :175-221 (ReconstOne)."""
    out = _host_e2e_pass(R, args)
    out["path"] = "pinned host memory, kernels in place over PCIe (xrs_*_host zero-copy)"
    prev = os.environ.get("XRS_HOST_ZC")
    os.environ["XRS_HOST_ZC"] = "0"  # read per call (codec.cpp host_zero_copy)
    try:
        dma = _host_e2e_pass(R, args)
    finally:
        if prev is None:
            del os.environ["XRS_HOST_ZC"]
        else:
            os.environ["XRS_HOST_ZC"] = prev
    dma["path"] = ("pinned host memory, hipMemcpy2DAsync H2D -> kernel -> D2H over three "
                   "streams in 64 MiB chunks (XRS_HOST_ZC=0)")
    out["dma"] = dma
    return out


def _host_e2e_pass(R: Rank, args):
    import ctypes

    import numpy as np

    torch, x, L = R.torch, R.x, R.xrs_amd.lib()
    out = {}
    for key, size, kind in (("encode_4k", ENC_S, "enc"), ("reconst_one_1m", REC_S, "rec")):
        stripe = (D + P) * size
        n = max(1, (args.host_mib << 20) // stripe)
        nbytes = n * stripe
        ptr = L.xrs_host_alloc(nbytes)
        if not ptr:
            raise RuntimeError("xrs_host_alloc failed")
        try:
            host = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(ptr))
            torch.from_numpy(host).copy_(R.random_bytes(nbytes, 0x4057 + R.w.rank))
            x.encode_host(ptr, size, size, stripe, n)
            if kind == "enc":
                fn = lambda i: x.encode_host(ptr, size, size, stripe, n)
                algo = n * (D + P) * size
            else:
                fn = lambda i: x.reconst_one_host(ptr, size, size, stripe, n, i % D)
                algo = n * 9 * size
            fn(0)
            secs = R.timed(fn, 3, 1)
            out[key] = {"stripes_per_rank": n, "bytes_per_call": algo,
                        "rank_gibps": [round(algo * 3 / t / GIB, 2) for t in secs],
                        "gibps": round(algo * 3 * R.w.world / max(secs) / GIB, 2)}
        finally:
            L.xrs_host_free(ptr)
    return out


XGMI_PLACEMENTS = {"half": lambda dev, ndev, i: dev if i % 2 == 0 else (dev + 1) % ndev,
                   "spread": lambda dev, ndev, i: (dev + i) % ndev}


def xgmi_need_plan(dev: int, ndev: int, k: int, size: int, n: int, a_need, b_need) -> dict:
    """Which need-set bytes of ReconstOne(k) (GetNeedVects, xrs.go:146-171;
    read set xrs.go:175-221) each placement puts on a peer GPU (no GPU call):
    the b-halves of the d - 1 surviving data vects, of parity d and of parity
    bi, and the a-halves of aNeed.  Per layout: the shards read, how many
    live on a peer, and the bytes the kernel on `dev` reads over xGMI per
    call (n stripes)."""
    half = size // 2
    halves = {}  # shard -> halves read per stripe
    for m in range(D):
        if m != k:
            halves[m] = halves.get(m, 0) + 1
    for b in b_need:
        halves[b] = halves.get(b, 0) + 1
    for a in a_need:
        halves[a] = halves.get(a, 0) + 1
    out = {}
    for name, place in XGMI_PLACEMENTS.items():
        remote = {i: c for i, c in halves.items() if place(dev, ndev, i) != dev}
        out[name] = {
            "need_set_shards": len(halves), "need_set_shards_remote": len(remote),
            "need_set_bytes": n * half * sum(halves.values()),
            "need_set_bytes_remote": n * half * sum(remote.values()),
            "gpus_read": sorted({place(dev, ndev, i) for i in halves}),
        }
    return out


def xgmi_repair(R: Rank, args):
    """Cross-GPU repair: rank 0 rebuilds data shard k of
    1 MiB stripes whose shards live on other GPUs, reading them over xGMI
    (xrs_reconst_one_shards after xrs_enable_peer_access), and checks the
    result bit for bit against the stored shard.  Two placements:
      * "half":   the odd-numbered shards on the next GPU;
      * "spread": shard i on GPU (device + i) mod (GPUs visible), i.e. a
                  stripe spread over the node, 2 shards per GPU at 8 GPUs.
    The rate is algorithmic bytes (9*S per stripe, xrs_test.go:565-572) over
    the call, next to the same rebuild from all-local shards.
    Semantics: xrs.go:175-221."""
    torch, x, s = R.torch, R.x, R.stream
    dev, ndev = R.dev_index, R.ndev
    # XRS_XGMI_SELF=1 on a one-GPU box: every "peer" is the same device (every
    # step but the xGMI reads themselves; tests/test_gpu_bench.py)
    for q in sorted({(dev + j) % ndev for j in range(1, D + P)} - {dev}):
        rc = R.xrs_amd.lib().xrs_enable_peer_access(dev, q)
        if rc != 0:
            return {"skipped": f"peer access {dev}->{q} unavailable (code {rc})"}
    n, size, k = args.xgmi_stripes, REC_S, 4
    col = n * size  # shard-major: shard i of stripe t at base + i*col + t*size
    local = R.random_bytes((D + P) * col, 0x961)
    x.encode_batched(local.data_ptr(), size, col, size, n, s)
    R.sync()
    expect = local[k * col:(k + 1) * col].clone()
    a_need, b_need = x.get_need_vects(k)
    plan = xgmi_need_plan(dev, ndev, k, size, n, a_need, b_need)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def rate(table):
        for _ in range(2):
            x.reconst_one_shards(table, size, size, n, k, s)
        reps = 10
        e0.record()
        for _ in range(reps):
            x.reconst_one_shards(table, size, size, n, k, s)
        e1.record()
        R.sync()
        return round(n * 9 * size / (e0.elapsed_time(e1) / reps / 1e3) / 1e9, 1)

    placements = {name: (lambda i, f=f: f(dev, ndev, i)) for name, f in XGMI_PLACEMENTS.items()}
    out = {"device": dev, "gpus_visible": ndev, "stripes": n, "vect_bytes": size, "k": k,
           "bytes_per_call": n * 9 * size, "layouts": {}}
    exact_all = True
    for name, place in placements.items():
        copies = {i: local[i * col:(i + 1) * col].to(f"cuda:{place(i)}")
                  for i in range(D + P) if i != k and (place(i) != dev or ndev == 1)}
        for q in range(ndev):
            torch.cuda.synchronize(q)
        table = [copies[i].data_ptr() if i in copies else local.data_ptr() + i * col
                 for i in range(D + P)]
        local[k * col:(k + 1) * col].zero_()
        x.reconst_one_shards(table, size, size, n, k, s)
        R.sync()
        exact = bool(torch.equal(local[k * col:(k + 1) * col], expect))
        gbs = rate(table)
        exact = exact and bool(torch.equal(local[k * col:(k + 1) * col], expect))
        exact_all = exact_all and exact
        out["layouts"][name] = dict(plan[name], gbs_algorithmic=gbs, bitexact=exact)
        del copies, table
        torch.cuda.empty_cache()
    out["gbs_all_local"] = rate([local.data_ptr() + i * col for i in range(D + P)])
    out["gbs_algorithmic"] = out["layouts"]["half"]["gbs_algorithmic"]
    out["need_set_bytes_remote"] = out["layouts"]["half"]["need_set_bytes_remote"]
    out["xgmi_bitexact"] = exact_all
    del local, expect
    torch.cuda.empty_cache()
    return out


def run_xgmi_child(args, device: int, ndev: int):
    """xgmi_repair in a child process (rank 0 only, other ranks wait at a
    barrier), so that a fault on the peer path cannot take the bench line
    with it; the child's JSON line (or its failure) becomes the key."""
    import subprocess

    if ndev < 2 and not os.environ.get("XRS_XGMI_SELF"):
        return {"skipped": f"{ndev} GPU visible to rank 0 (cross-GPU repair needs two)"}
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT")}
    cmd = [sys.executable, os.path.abspath(__file__), "--xgmi-child", str(device),
           "--xgmi-stripes", str(args.xgmi_stripes)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=150, env=env)
    except subprocess.TimeoutExpired:
        return {"error": "timed out after 150 s"}
    except OSError as e:
        return {"error": f"could not start the probe: {e}"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"exit {r.returncode}", "stderr_tail": r.stderr[-800:]}
    return json.loads(lines[-1])


def per_stripe_queue(args):
    """The reference's call pattern (one Encode per stripe, xrs_test.go:498-521)
    from T concurrent caller threads through the batching queue
    (xrs_queue_encode, xrs_amd/csrc/queue.cpp): tools/sync_bench, a C++ child
    process, 2 s per caller count, host-resident 12+4 stripes of 4 KiB.  Rate
    in the reference's bytes (16 * S per stripe), PCIe-inclusive; not part of
    `value`."""
    import subprocess

    exe = os.path.join(ROOT, "tools", "sync_bench")
    if not os.path.exists(exe):
        return {"skipped": "tools/sync_bench not built (build() makes it)"}
    def child(mode, size=4096, window=None, callers=None):
        cmd = [exe, str(size), mode] + (["50"] if mode.startswith("queue") else []) + (
            [str(window)] if window else []) + [str(t) for t in (callers or args.queue_callers)]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
        except subprocess.TimeoutExpired:
            return None, {"error": "timed out after 120 s"}
        lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not lines:
            return None, {"error": f"exit {r.returncode}", "stdout_tail": r.stdout[-400:]}
        return lines, None

    lines, err = child("queue")
    out = err or {"api": "xrs_queue_encode", "vect_bytes": 4096, "codec": "12+4",
                  "by_callers": {str(x["threads"]): {k: x[k] for k in (
                      "gibps", "stripes_per_s", "stripes_per_batch", "run_us_per_batch",
                      "wait_us_per_batch", "cpu_cores", "cpu_seconds_per_gib") if k in x}
                      for x in lines},
                  "cpu_note": ("cpu_cores = process CPU time (callers' copies + the queue's "
                               "launcher and completion threads) / wall time")}
    # the same callers with their vects in registered memory (xrs_host_alloc:
    # the cgo shim's pinned buffer pool): no CPU copy through staging, one
    # indirect-row launch per batch in place (queue.cpp table mode)
    lines, err = child("queuereg")
    out["registered"] = err or {"by_callers": {str(x["threads"]): {k: x[k] for k in (
        "gibps", "stripes_per_s", "stripes_per_batch", "run_us_per_batch", "wait_us_per_batch",
        "cpu_cores", "cpu_seconds_per_gib") if k in x} for x in lines}}
    # the plain drop-in call (xrs_encode per stripe) from the same number of
    # threads on ONE codec: contended calls batch through the codec's queue
    def plain(mode):
        lines, err = child(mode)
        return err or {x["api"].split()[0]: {str(x["threads"]): {k: x[k] for k in (
            "gibps", "calls_per_s", "cpu_cores", "cpu_seconds_per_gib") if k in x}}
            for x in lines}
    out["plain_api"] = plain("syncmt")
    out["plain_api_registered"] = plain("syncmtreg")
    # 64 KiB vects (1 MiB per stripe), where the callers' copies dominate the
    # CPU cost: the queue with plain and with registered vects
    big = {}
    for name, mode in (("plain", "queue"), ("registered", "queuereg")):
        lines, err = child(mode, 65536)
        big[name] = err or {str(x["threads"]): {k: x[k] for k in (
            "gibps", "stripes_per_batch", "run_us_per_batch", "cpu_cores", "cpu_seconds_per_gib")
            if k in x} for x in lines}
    out["queue_64k"] = big
    # the asynchronous calls (xrs_queue_submit_encode + xrs_queue_wait): each
    # caller thread keeps a window of stripes in flight -- one cgo call site
    # with k stripes outstanding instead of k blocked OS threads
    asy = {"api": "xrs_queue_submit_encode + xrs_queue_wait", "window": args.async_window}
    for name, mode in (("plain", "queueasync"), ("registered", "queueasyncreg")):
        lines, err = child(mode, 4096, args.async_window, args.async_callers)
        asy[name] = err or {str(x["threads"]): {k: x[k] for k in (
            "gibps", "stripes_per_batch", "run_us_per_batch", "busy_returns", "cpu_cores",
            "cpu_seconds_per_gib") if k in x} for x in lines}
    out["async_4k"] = asy
    return out


def xgmi_child(args) -> int:
    R = Rank(xdist.World(0, 1, args.xgmi_child, False), "none")
    print(json.dumps(xgmi_repair(R, args)), flush=True)
    return 0


def run_rank(args, w):
    # The bracket around a timed region is a host barrier plus a gather of
    # per-rank times: no byte of shard data crosses ranks, so no RCCL
    # communicator is needed (gloo over 127.0.0.1).  XRS_DIST_BACKEND=nccl
    # runs the same bracket over RCCL instead.
    backend = os.environ.get("XRS_DIST_BACKEND", "gloo")
    R = Rank(w, backend)
    launches, step_bytes, rank_seconds, kernels, strides, samples = headline(R, args)
    elapsed_max = max(rank_seconds)
    value = w.world * args.steps * step_bytes / elapsed_max / GIB

    dom_key = max(kernels, key=lambda k: kernels[k]["ms"])
    dom = kernels[dom_key]
    traffic, traffic_source = pmc_traffic(dom_key, dom["kernel"], R.xrs_amd.LIB_PATH)
    roofline = {
        "bound": "hbm", "kernel": dom["kernel"], "launch": dom_key,
        "achieved": dom["achieved_gbs"],
        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(dom["achieved_gbs"] / HBM_PEAK_GBS, 4),
        "traffic": traffic, "traffic_source": traffic_source,
        "algorithmic_bytes_per_launch": dom["bytes_per_launch"],
        # the north star's "HBM-read roofline": read bytes only over the same
        # peak (DESIGN.md §5 explains why 0.70 of it is out of reach for a
        # 12:4 read:write pattern)
        "read_achieved": dom["read_only_gbs"],
        "read_frac": dom["read_frac"],
    }

    c5 = None
    if args.config5_stripes > 0:
        c5 = config5(R, args)
    c4 = None
    if args.config4_stripes > 0:
        c4, c4_samples = config4(R, args)
        if not args.no_parity:
            samples += c4_samples
    he = host_e2e(R, args) if args.host_mib > 0 else None
    pq = None
    if w.rank == 0 and w.world == 1 and args.queue_callers:
        log("per-stripe calls through the batching queue ...")
        pq = per_stripe_queue(args)
    xg = None
    if args.xgmi_stripes > 0:
        xdist.barrier()
        if w.rank == 0:
            xg = run_xgmi_child(args, R.dev_index, R.ndev)
        xdist.barrier()

    # Checker leg (untimed): the oracle on every rank's parity samples, then
    # the CPU baseline on rank 0 at N = 1.
    parity = None
    if samples:
        log("oracle parity of the sampled stripes ...")
        mine = oracle_parity(samples)
        oks = [v > 0.5 for v in xdist.gather_seconds(
            1.0 if all(c["bitexact"] for c in mine["cases"]) else 0.0, R.tdev)]
        parity = dict(mine, all_ranks=oks, bitexact=all(oks))
        del samples
    cpu = None
    if w.rank == 0 and w.world == 1 and not args.no_cpu_baseline:
        log("timing CPU baseline ...")
        cpu = cpu_baseline(args.cpu_seconds, {l[0]: l[2] for l in launches})

    if w.rank == 0:
        enc_shard, rec_shard = strides
        out = {
            "metric": "Encode + 1-lost Reconstruct GiB/s (device-resident), 12+4 @ 4KiB/1MiB",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": w.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (uniform random bytes generated on device, seeded per rank)",
            "config": {
                "workload": (f"12+4 Encode + ReconstOne (k = step mod 12) of {args.enc_stripes} "
                             f"stripes @ 4 KiB and of {args.rec_stripes} stripes @ 1 MiB, per GPU "
                             f"per step"),
                "data_shards": D, "parity_shards": P,
                "encode_vect_bytes": ENC_S, "encode_stripes_per_gpu": args.enc_stripes,
                "reconst_vect_bytes": REC_S, "reconst_stripes_per_gpu": args.rec_stripes,
                "encode_shard_stride": enc_shard, "reconst_shard_stride": rec_shard,
                "parallelism": f"stripe split x{w.world}, no collective",
            },
            "library": library_info(R.xrs_amd),
            "rank_seconds": [round(v, 6) for v in rank_seconds],
            "rank_devices": R.rank_devices,
            "shared_gpu": R.shared_gpu,
            "kernels": kernels,
            "roofline": roofline,
            "parity": parity,
            "cpu_baseline": cpu,
            "config4": c4,
            "config5": c5,
            "host_e2e": he,
            "per_stripe_queue": pq,
            "xgmi_repair": xg,
        }
        print(json.dumps(out), flush=True)
    xdist.finalize()
    return 0


def main(argv=None):
    args = parse_args(argv)
    if args.xgmi_child is not None:  # rank 0's isolated cross-GPU repair probe
        return xgmi_child(args)
    try:
        w = xdist.resolve_world(args.gpus)
    except xdist.WorldMismatch as e:
        log(f"bench.py: {e}")
        return 2
    if w.world > 1 and not w.launched:
        # `python bench.py --gpus N` without torchrun: start the N ranks here,
        # before this process makes any GPU call, and exit with their status.
        argv = sys.argv[1:] if argv is None else list(argv)
        return xdist.launch_local(w.world, [sys.executable, os.path.abspath(__file__)] + argv)
    try:
        return run_rank(args, w)
    except xdist.SharedDevice as e:
        log(f"bench.py: {e}")
        return 3


if __name__ == "__main__":
    sys.exit(main())
