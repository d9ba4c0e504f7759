"""Multi-rank tests (CPU, gloo, world size 2-3) of the harness bench.py runs
on N GPUs (xrs_amd/dist.py): the rank layout and its --gpus check, the
self-launch of `bench.py --gpus N`, the stripe split and the barrier +
per-rank time bracket.  The per-rank compute is the CPU oracle here (the GPU
box runs the kernels; 8-GPU runs are the driver's)."""
import json
import os
import subprocess
import sys

import pytest

from xrs_amd import dist as xdist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "_rank_worker.py")


def test_stripe_range_partitions():
    for n in (0, 1, 7, 8, 65536, 65537):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                s, c = xdist.stripe_range(n, r, world)
                seen.extend(range(s, s + c))
            assert seen == list(range(n))
    with pytest.raises(ValueError):
        xdist.stripe_range(8, 2, 2)
    # config 5: 65,536 stripes over 8 GPUs = 8,192 each
    assert [xdist.stripe_range(65536, r, 8)[1] for r in range(8)] == [8192] * 8


def test_resolve_world():
    w = xdist.resolve_world(None, env={})
    assert (w.rank, w.world, w.launched) == (0, 1, False)
    w = xdist.resolve_world(8, env={})
    assert (w.rank, w.world, w.launched) == (0, 8, False)  # bench.py launches the 8 ranks
    env = {"WORLD_SIZE": "4", "RANK": "3", "LOCAL_RANK": "3"}
    w = xdist.resolve_world(4, env=env)
    assert (w.rank, w.world, w.local, w.launched) == (3, 4, 3, True)
    assert xdist.resolve_world(None, env=env).world == 4
    with pytest.raises(xdist.WorldMismatch):
        xdist.resolve_world(2, env=env)
    with pytest.raises(xdist.WorldMismatch):
        xdist.resolve_world(0, env={})


def test_bench_gpus_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode == 2
    assert "--gpus 2" in r.stderr and "WORLD_SIZE=4" in r.stderr
    assert not r.stdout.strip()


def test_bench_self_launch_starts_n_ranks_without_gpu():
    """`bench.py --gpus 2` without a launcher starts two rank processes; on
    this GPU-less host each rank fails loudly (no CPU fallback) and the parent
    returns a non-zero status."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "1"], capture_output=True, text=True, timeout=180, env=env,
                       cwd=ROOT)
    assert r.returncode != 0
    assert "needs a GPU" in r.stderr
    assert not r.stdout.strip()


@pytest.mark.parametrize("world,n_stripes", [(2, 64), (2, 65), (3, 65)])
def test_launch_local_split_encode_gloo(tmp_path, world, n_stripes):
    rc = xdist.launch_local(world, [sys.executable, WORKER, str(tmp_path), str(n_stripes), "4096"],
                            timeout=240)
    assert rc == 0
    res = json.loads((tmp_path / "result.json").read_text())
    assert res["ok"] and res["world"] == world
    assert len(res["rank_seconds"]) == world and min(res["rank_seconds"]) > 0
    assert len(res["region_seconds"]) == world
    assert sum(res["counts"]) == n_stripes


def test_rank_stdout_carries_no_gloo_noise(tmp_path):
    """gloo's C++ side prints "[Gloo] Rank r is connected to ..." on stdout
    while a group connects; xdist.init sends it to stderr, so rank 0's stdout
    holds only what the program prints (bench.py: its one JSON line)."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from xrs_amd import dist as x\n"
            "sys.exit(x.launch_local(2, [sys.executable, %r, %r, '16', '64'], timeout=200))\n"
            % (ROOT, WORKER, str(tmp_path)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Gloo" not in r.stdout, r.stdout
    assert json.loads((tmp_path / "result.json").read_text())["ok"]


def test_launch_local_propagates_a_failed_rank(tmp_path):
    rc = xdist.launch_local(2, [sys.executable, WORKER, str(tmp_path), "8", "64", "1"],
                            timeout=240)
    assert rc == 3
    assert not (tmp_path / "result.json").exists()


DEV_WORKER = os.path.join(ROOT, "tests", "_device_worker.py")


def test_check_distinct_devices():
    a = {"rank": 0, "pci": "0000:05:00"}
    b = {"rank": 1, "pci": "0000:15:00"}
    assert xdist.check_distinct_devices([a, b], rehearsal=False) is False
    same = dict(b, pci=a["pci"])
    with pytest.raises(xdist.SharedDevice, match="ranks 0 and 1"):
        xdist.check_distinct_devices([a, same], rehearsal=False)
    assert xdist.check_distinct_devices([a, same], rehearsal=True) is True
    assert xdist.rehearsal_env({"XRS_REHEARSAL": "1"}) and not xdist.rehearsal_env({})
    assert not xdist.rehearsal_env({"XRS_REHEARSAL": "0"})


@pytest.mark.parametrize("pcis,rehearsal,rc,shared", [
    ("0000:05:00,0000:15:00", False, 0, False),     # two GPUs: fine
    ("0000:05:00,0000:05:00", False, 3, None),      # one card, no label: refused
    ("0000:05:00,0000:05:00", True, 0, True),       # labelled rehearsal
])
def test_rank_devices_gloo(tmp_path, pcis, rehearsal, rc, shared):
    """The start-up gather of every rank's GPU over gloo, world size 2: a
    layout where two ranks share a card exits 3 (bench.py's status) unless
    XRS_REHEARSAL=1, and then says shared."""
    env = dict(os.environ, XRS_TEST_PCI=pcis)
    env.pop("XRS_REHEARSAL", None)
    if rehearsal:
        env["XRS_REHEARSAL"] = "1"
    got = xdist.launch_local(2, [sys.executable, DEV_WORKER, str(tmp_path)], env=env, timeout=200)
    assert got == rc
    if rc == 0:
        res = json.loads((tmp_path / "result.json").read_text())
        assert res["shared"] is shared
        assert [d["pci"] for d in res["devices"]] == pcis.split(",")
    else:
        assert "same GPU" in (tmp_path / "refused.txt").read_text()


def test_launch_local_sigterm_stops_the_ranks(tmp_path):
    """SIGTERM to the launching parent stops every rank it started (a
    driver's time limit must not leave ranks holding GPUs)."""
    import signal
    import time
    rank = tmp_path / "rank.py"
    rank.write_text("import os, sys, time\n"
                    "d = sys.argv[1]\n"
                    "open(os.path.join(d, 'pid' + os.environ['RANK']), 'w').write(str(os.getpid()))\n"
                    "time.sleep(600)\n")
    parent = tmp_path / "parent.py"
    parent.write_text("import sys\n"
                      f"sys.path.insert(0, {ROOT!r})\n"
                      "from xrs_amd import dist as xdist\n"
                      f"sys.exit(xdist.launch_local(2, [sys.executable, {str(rank)!r}, {str(tmp_path)!r}]))\n")
    proc = subprocess.Popen([sys.executable, str(parent)])
    deadline = time.monotonic() + 120
    while len(list(tmp_path.glob("pid*"))) < 2 and time.monotonic() < deadline:
        time.sleep(0.1)
    time.sleep(0.2)
    pids = [int(p.read_text()) for p in tmp_path.glob("pid*")]
    assert len(pids) == 2
    proc.send_signal(signal.SIGTERM)
    assert proc.wait(timeout=60) != 0
    for pid in pids:
        for _ in range(100):
            try:
                os.kill(pid, 0)
            except ProcessLookupError:
                break
            time.sleep(0.1)
        else:
            raise AssertionError(f"rank {pid} still running")


def test_bench_multi_gpu_keys_8_ranks(tmp_path):
    """The keys the driver's 8-GPU bench line must carry, built by bench.py's
    own split / placement functions (config5_plan, xgmi_need_plan) and the
    start-up device gather, over 8 gloo ranks on CPU
    (tests/_bench_plan_worker.py): config 5 as an 8-way split of 65,536
    stripes (8,192 per GPU, contiguous ranges), one rank_devices entry per
    rank on distinct GPUs, and xgmi_repair's need-set bytes read from peers
    (ReconstOne's need set, xrs.go:146-221: 8 S of 9 S per stripe read)."""
    worker = os.path.join(ROOT, "tests", "_bench_plan_worker.py")
    rc = xdist.launch_local(8, [sys.executable, worker, str(tmp_path)], timeout=300)
    assert rc == 0
    line = json.loads((tmp_path / "line.json").read_text())
    assert line["n_gpus"] == 8 and line["shared_gpu"] is False
    assert [d["rank"] for d in line["rank_devices"]] == list(range(8))
    assert len({d["pci"] for d in line["rank_devices"]}) == 8
    c5 = line["config5"]
    assert c5["stripes_total"] == 65536 and c5["stripes_per_rank"] == 8192
    assert c5["rank_ranges"] == [[8192 * r, 8192] for r in range(8)]
    xg = line["xgmi_repair"]
    half, spread = xg["layouts"]["half"], xg["layouts"]["spread"]
    S = 1 << 20
    # every layout reads the same need set: 8 S per stripe over 64 stripes
    assert half["need_set_bytes"] == spread["need_set_bytes"] == 64 * 8 * S
    assert half["need_set_shards"] == 13  # 11 data + parity 12 + parity bi
    # "half": odd shards on GPU 1; "spread": shard i on GPU i mod 8 (shards 0
    # and 8 of the need set stay on GPU 0)
    assert 0 < half["need_set_bytes_remote"] < half["need_set_bytes"]
    assert half["gpus_read"] == [0, 1]
    assert spread["need_set_shards_remote"] == spread["need_set_shards"] - 2
    assert len(spread["gpus_read"]) == 8
    assert xg["need_set_bytes_remote"] == half["need_set_bytes_remote"]
