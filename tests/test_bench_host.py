"""CPU tests of bench.py's host-side pieces that need no GPU: the
per_stripe_queue key's child-process protocol (tools/sync_bench output
parsing, a missing or failing binary)."""
import importlib.util
import os
import stat
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _fake_sync_bench(tmp_path, body):
    tools = tmp_path / "tools"
    tools.mkdir()
    exe = tools / "sync_bench"
    exe.write_text("#!/bin/sh\n" + body)
    exe.chmod(exe.stat().st_mode | stat.S_IEXEC)


def test_per_stripe_queue_parses_both_children(tmp_path, monkeypatch):
    bench = _bench()
    _fake_sync_bench(tmp_path, """case "$2" in
queue) echo '{"api": "xrs_queue_encode", "vect_bytes": 4096, "threads": 32, "stripes_per_s": 480000, "gibps": 29.3, "batches": 1, "stripes_per_batch": 8.0, "run_us_per_batch": 38.0, "wait_us_per_batch": 15.0}' ;;
syncmt) echo '{"api": "xrs_encode (per-stripe, shared codec)", "vect_bytes": 4096, "threads": 32, "calls_per_s": 500000, "gibps": 30.5}'
        echo '{"api": "xrs_update (per-stripe, shared codec)", "vect_bytes": 4096, "threads": 32, "calls_per_s": 600000, "gibps": 22.9}' ;;
queueasyncreg) [ "$3" = 50 ] && [ "$4" = 16 ] && [ "$5" = 4 ] && echo '{"api": "xrs_queue_submit_encode + xrs_queue_wait", "vect_bytes": 4096, "threads": 4, "window": 16, "gibps": 44.0, "busy_returns": 0, "cpu_cores": 3.1, "cpu_seconds_per_gib": 0.07}' ;;
esac
""")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    out = bench.per_stripe_queue(types.SimpleNamespace(queue_callers=[32], async_window=16,
                                                       async_callers=[4]))
    assert out["by_callers"]["32"]["gibps"] == 29.3
    # the asynchronous leg: WAIT_US 50, the window, then the caller counts
    assert out["async_4k"]["registered"]["4"]["gibps"] == 44.0
    assert out["async_4k"]["window"] == 16
    assert out["by_callers"]["32"]["stripes_per_batch"] == 8.0
    assert out["plain_api"]["xrs_encode"]["32"]["gibps"] == 30.5
    assert out["plain_api"]["xrs_update"]["32"]["calls_per_s"] == 600000


def test_per_stripe_queue_missing_or_failing_binary(tmp_path, monkeypatch):
    bench = _bench()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    ns = types.SimpleNamespace(queue_callers=[32], async_window=16, async_callers=[4])
    assert "skipped" in bench.per_stripe_queue(ns)
    _fake_sync_bench(tmp_path, "echo 'queue call failed: 9'; exit 5\n")
    out = bench.per_stripe_queue(ns)
    assert out["error"] == "exit 5" and "queue call failed" in out["stdout_tail"]
    assert out["plain_api"]["error"] == "exit 5"
