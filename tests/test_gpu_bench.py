"""GPU tests of bench.py's driver contract: one JSON line with the required
keys, at N=1 and at N=2 (two ranks through torch.distributed.run; on the
one-GPU box they share cuda:0; the bracket runs over gloo, bench.py's default
(RCCL refuses two ranks on one device, so XRS_DIST_BACKEND=nccl needs two GPUs))."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--steps", "3", "--warmup", "1", "--enc-stripes", "2048", "--rec-stripes", "16",
         "--no-cpu-baseline", "--config5-stripes", "64", "--config5-steps", "2", "--host-mib", "32",
         "--xgmi-stripes", "4", "--ramp-seconds", "0.3", "--config4-stripes", "4",
         "--config4-steps", "2"]
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
        "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline",
        "cpu_baseline", "parity", "rank_devices", "shared_gpu", "config4", "library"}
PARITY_KEYS = ("encode_4k", "reconst_one_4k", "encode_1m", "reconst_one_1m", "config4_update",
               "config4_replace4")


def _check_parity(j):
    """The line's oracle parity leg: every headline launch bit-exact on its
    sampled stripes (first / middle / last), ReconstOne at two k, and config
    4's Update and Replace(4) on their first / last stripes; the measured
    library is the tree's (source digest, xrs_version())."""
    par = j["parity"]
    assert par["oracle"] == "oracle/xrs_oracle.c"
    assert all(par[k] is True for k in PARITY_KEYS), par
    assert par["bitexact"] is True and all(par["all_ranks"])
    assert len(par["cases"]) == 8 and all(c["bitexact"] for c in par["cases"])
    assert j["library"]["built_from_tree"] is True, j["library"]
    c4 = j["config4"]
    assert c4["update"]["gibps"] > 0 and c4["replace4"]["gibps"] > 0


def _line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_one_gpu_contract():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + SMALL,
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    j = _line(r.stdout)
    assert KEYS <= set(j)
    assert j["n_gpus"] == 1 and j["steps"] == 3 and j["value"] > 0
    assert j["roofline"]["bound"] == "hbm" and 0 < j["roofline"]["frac"] < 1
    assert set(j["kernels"]) == {"encode_4k", "reconst_one_4k", "encode_1m", "reconst_one_1m"}
    _check_parity(j)
    assert j["shared_gpu"] is False and len(j["rank_devices"]) == 1
    c5 = j["config5"]
    assert c5["stripes_total"] == 64 and c5["stripes_per_rank"] == 64 and c5["roundtrip_ok"]
    assert len(c5["encode"]["rank_seconds"]) == 1 and c5["gibps"] > 0
    assert set(j["host_e2e"]) >= {"encode_4k", "reconst_one_1m", "dma"}
    assert set(j["host_e2e"]["dma"]) >= {"encode_4k", "reconst_one_1m", "path"}
    assert j["host_e2e"]["dma"]["encode_4k"]["gibps"] > 0
    xg = j["xgmi_repair"]
    assert ("skipped" in xg) or xg["xgmi_bitexact"], xg


def test_bench_xgmi_child_self_peer():
    """The cross-GPU repair probe end to end on one card (XRS_XGMI_SELF: the
    "peer" shards are a second allocation on the same device), so the path
    the driver's multi-GPU run takes is exercised here."""
    env = dict(os.environ, XRS_XGMI_SELF="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + SMALL
                       + ["--config5-stripes", "0", "--host-mib", "0"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    xg = _line(r.stdout)["xgmi_repair"]
    assert xg["xgmi_bitexact"] is True, xg
    assert xg["gbs_algorithmic"] > 0 and xg["gbs_all_local"] > 0


def test_bench_two_ranks_refused_on_one_card():
    """Two ranks on a one-GPU box without XRS_REHEARSAL: bench.py refuses
    (exit 3) instead of printing a line that claims two GPUs."""
    import torch
    if torch.cuda.device_count() > 1:
        pytest.skip("two GPUs visible: the ranks would not share a card")
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "XRS_REHEARSAL")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL,
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 3, r.stderr[-3000:]
    assert "same GPU" in r.stderr and not r.stdout.strip()


def test_bench_two_ranks_contract():
    env = dict(os.environ, XRS_REHEARSAL="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    j = _line(r.stdout)
    assert KEYS <= set(j)
    assert j["n_gpus"] == 2 and j["scaling"] == "weak" and j["value"] > 0
    assert j["cpu_baseline"] is None  # rank 0 at N=1 only
    assert len(j["rank_seconds"]) == 2 and min(j["rank_seconds"]) > 0
    assert abs(j["ms_per_step"] * j["steps"] / 1e3 - max(j["rank_seconds"])) < 1e-3
    c5 = j["config5"]
    assert c5["stripes_total"] == 128 and c5["roundtrip_ok"] and len(c5["roundtrip_ok_ranks"]) == 2
    assert len(j["config5"]["reconst_one"]["rank_seconds"]) == 2
    assert len(j["host_e2e"]["encode_4k"]["rank_gibps"]) == 2
    _check_parity(j)
    assert len(j["rank_devices"]) == 2
    assert j["shared_gpu"] is (torch_device_count() < 2)


def torch_device_count():
    import torch
    return torch.cuda.device_count()


def test_bench_self_launch_two_ranks():
    """`bench.py --gpus 2` without torchrun starts its two ranks itself (the
    form the driver may use); on a one-GPU box they share cuda:0 over gloo."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["XRS_REHEARSAL"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL,
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    j = _line(r.stdout)
    assert j["n_gpus"] == 2 and len(j["rank_seconds"]) == 2 and min(j["rank_seconds"]) > 0
    assert j["config5"]["stripes_total"] == 128
    xg = j["xgmi_repair"]
    assert ("skipped" in xg) or xg["xgmi_bitexact"]
