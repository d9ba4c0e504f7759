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
esac
""")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    out = bench.per_stripe_queue(types.SimpleNamespace(queue_callers=[32]))
    assert out["by_callers"]["32"]["gibps"] == 29.3
    assert out["by_callers"]["32"]["stripes_per_batch"] == 8.0
    assert out["plain_api"]["xrs_encode"]["32"]["gibps"] == 30.5
    assert out["plain_api"]["xrs_update"]["32"]["calls_per_s"] == 600000


def test_per_stripe_queue_missing_or_failing_binary(tmp_path, monkeypatch):
    bench = _bench()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert "skipped" in bench.per_stripe_queue(types.SimpleNamespace(queue_callers=[32]))
    _fake_sync_bench(tmp_path, "echo 'queue call failed: 9'; exit 5\n")
    out = bench.per_stripe_queue(types.SimpleNamespace(queue_callers=[32]))
    assert out["error"] == "exit 5" and "queue call failed" in out["stdout_tail"]
    assert out["plain_api"]["error"] == "exit 5"
