"""pytest plugin for tools/r06_fault_probe.sh (diagnosis of the intermittent
illegal-address fault; never loaded by the suite itself).

It records every host range the tests pin through the C ABI
(xrs_host_register / _unregister / _alloc / _free, with the test that made and
released it), and for every D2H `.cpu()` of a device tensor it allocates the
pageable destination first and asks HIP (hipPointerGetAttributes) what it
knows about it before copying.  A pageable buffer the runtime still reports as
known memory, or one lying on a range the tests pinned earlier, is logged as
SUSPECT.  After each test it also probes fresh pageable buffers of the sizes
test_gpu_shards.py copies into.  Events go to gpurun_out/r06_fault_probe.log.
"""
import ctypes
import os

import pytest

_OUT = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "r06_fault_probe.log")
_log = None
_ranges = []  # [kind, lo, hi, made_by, released_by]
_cur = ["-"]
_hip = None
_stats = {"cpu": 0, "suspect": 0, "fresh": 0}
_SIZES = [4096, 79310, 1228800, 6 << 20, 16 << 20]


class _Attr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


def _w(msg):
    _log.write(msg + "\n")
    _log.flush()


def _attrs(p):
    a = _Attr()
    rc = _hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(p))
    _hip.hipGetLastError()  # a pageable pointer sets an error; torch must not see it
    return rc, a.type, a.devicePointer or 0, a.hostPointer or 0, a.allocationFlags


def _hits(p, n):
    return [(k, hex(lo), hi - lo, mk, rel) for k, lo, hi, mk, rel in _ranges if lo < p + n and p < hi]


def _probe(p, n, what):
    rc, ty, dp, hp, fl = _attrs(p)
    hits = _hits(p, n)
    bad = rc == 0 or hits
    if bad:
        _stats["suspect"] += 1
        _w(f"SUSPECT {what} {p:#x}+{n} attr rc={rc} type={ty} dev={dp:#x} host={hp:#x} flags={fl:#x} "
           f"overlaps={hits} in {_cur[0]}")
    return bad


def _install():
    global _hip, _log
    if _log is not None:
        return
    import torch

    import xrs_amd
    os.makedirs(os.path.dirname(_OUT), exist_ok=True)
    _log = open(_OUT, "w")
    rts = xrs_amd.hip_runtimes()
    _w(f"hip runtimes mapped: {rts}")
    _hip = ctypes.CDLL(rts[0])
    _hip.hipPointerGetAttributes.restype = ctypes.c_int
    _hip.hipGetLastError.restype = ctypes.c_int
    L = xrs_amd.lib()
    reg, unreg, alloc, free = L.xrs_host_register, L.xrs_host_unregister, L.xrs_host_alloc, L.xrs_host_free

    def _val(p):
        return p.value if isinstance(p, ctypes.c_void_p) else int(p or 0)

    def w_reg(p, n):
        rc = reg(p, n)
        lo = _val(p)
        _ranges.append(["register", lo, lo + int(n), _cur[0], None])
        return rc

    def w_unreg(p):
        rc = unreg(p)
        lo = _val(p)
        for r in reversed(_ranges):
            if r[0] == "register" and r[1] == lo and r[4] is None:
                r[4] = _cur[0]
                break
        return rc

    def w_alloc(n):
        p = alloc(n)
        if p:
            _ranges.append(["alloc", int(p), int(p) + int(n), _cur[0], None])
        return p

    def w_free(p):
        lo = _val(p)
        for r in reversed(_ranges):
            if r[0] == "alloc" and r[1] == lo and r[4] is None:
                r[4] = _cur[0]
                break
        return free(p)

    L.xrs_host_register, L.xrs_host_unregister = w_reg, w_unreg
    L.xrs_host_alloc, L.xrs_host_free = w_alloc, w_free
    orig_cpu = torch.Tensor.cpu

    def probe_cpu(self, *a, **k):
        if not (self.is_cuda and not a and not k):
            return orig_cpu(self, *a, **k)
        dst = torch.empty(self.shape, dtype=self.dtype)
        p, n = dst.data_ptr(), dst.numel() * dst.element_size()
        _stats["cpu"] += 1
        bad = _probe(p, n, "cpu-dst")
        if "test_gpu_shards" in _cur[0]:
            rc, ty, dp, hp, fl = _attrs(self.data_ptr())
            _w(f"shards copy {self.data_ptr():#x} (attr rc={rc} type={ty}) -> {p:#x}+{n} "
               f"{'SUSPECT' if bad else 'clean'} in {_cur[0]}")
        try:
            dst.copy_(self)
        except Exception as e:  # noqa: BLE001
            _w(f"COPY FAILED {self.data_ptr():#x} -> {p:#x}+{n}: {e!r} in {_cur[0]}")
            raise
        return dst

    torch.Tensor.cpu = probe_cpu


@pytest.hookimpl(tryfirst=True)
def pytest_runtest_setup(item):
    _install()
    _cur[0] = item.nodeid


def pytest_runtest_teardown(item):
    import torch
    held = []
    for n in _SIZES:
        t = torch.empty(n, dtype=torch.uint8)
        held.append(t)
        _stats["fresh"] += 1
        _probe(t.data_ptr(), n, "fresh")
    del held


def pytest_sessionfinish(session):
    if _log is not None:
        live = [r for r in _ranges if r[4] is None]
        _w(f"end: {_stats}, ranges pinned {len(_ranges)}, never released {len(live)}: {live[:20]}")
        _log.close()
