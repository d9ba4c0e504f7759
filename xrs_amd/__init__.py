"""xrs_amd -- MI355X-native X-Reed-Solomon codec (host mirror of templexxx/xrs).

Python mirror of the Go ``*XRS`` method set (/root/reference/xrs.go) over the
C ABI of ``libxrs_hip.so`` (include/xrs_hip.h).  Every byte of shard arithmetic
runs in the gfx950 kernels of that library; this module only marshals
arguments.  There is no CPU fallback: if the library is missing, importing
this package raises.

    x = XRS(12, 4)                 # xrs.go:55 New
    x.encode(vects)                # xrs.go:103 Encode (host buffers, in place)
    x.reconst(vects, dp_has, need) # xrs.go:236 Reconst
    x.encode_batched(ptr, size, shard_stride, stripe_stride, n_stripes, stream)
"""
from __future__ import annotations

import ctypes
import os
import threading

__all__ = ["XRS", "XRSGroup", "XRSQueue", "XRSError", "lib", "LIB_PATH", "batch_strides", "batch_layout",
           "hip_runtimes", "source_hash", "version", "library_source_hash",
           "trace_kernels", "traced_kernels"]

_HERE = os.path.dirname(os.path.abspath(__file__))
# XRS_LIB: an alternative build of the library (A/B experiments only).
LIB_PATH = os.environ.get("XRS_LIB") or os.path.join(_HERE, "libxrs_hip.so")

XRS_ERR_SIZE_NOT_EVEN = -2
XRS_ERR_ILLEGAL_DATA_INDEX = -3
XRS_ERR_ILLEGAL_VECTS = -4
XRS_ERR_INVALID_ARG = -9
XRS_ERR_BUSY = -11  # xrs_queue_submit_*: no staging batch free (nothing staged)


class XRSError(Exception):
    """An error returned by the codec; ``str()`` is the Go message text."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


def hip_runtimes() -> list:
    """Distinct libamdhip64 files mapped into this process (should be one)."""
    try:
        with open("/proc/self/maps") as f:
            return sorted({ln.split()[-1] for ln in f if "libamdhip64" in ln})
    except OSError:
        return []


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"xrs_amd: {LIB_PATH} is not built (run __graft_entry__.build() or "
            "make -C xrs_amd/csrc); there is no CPU fallback")
    # One HIP runtime per process.  PyTorch-ROCm bundles its own
    # libamdhip64 (soname libamdhip64.so.7) and links it by the unversioned
    # name: loaded first, it also satisfies this library's dependency; loaded
    # second, the loader would map a second runtime next to /opt/rocm's, and
    # device pointers, streams and events would belong to different runtimes.
    # So torch, when installed, is loaded before the codec library.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    if len(hip_runtimes()) > 1:
        raise ImportError(f"xrs_amd: two HIP runtimes in this process: {hip_runtimes()}")
    I, Z, P = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p
    IP = ctypes.POINTER(ctypes.c_int)
    PP = ctypes.POINTER(ctypes.c_void_p)
    sig = {
        "xrs_strerror": ([I], ctypes.c_char_p),
        "xrs_format_error": ([I, ctypes.c_longlong, ctypes.c_char_p, Z], I),
        "xrs_version": ([], ctypes.c_char_p),
        "xrs_trace_kernels": ([I], I),
        "xrs_traced_kernels": ([ctypes.c_char_p, Z], Z),
        "xrs_new": ([I, I, ctypes.POINTER(P)], I),
        "xrs_free": ([P], None),
        "xrs_data_num": ([P], I),
        "xrs_parity_num": ([P], I),
        "xrs_gen_matrix": ([P, P, Z], I),
        "xrs_xorset": ([P, I, IP, I, IP], I),
        "xrs_get_need_vects": ([P, I, IP, IP, IP], I),
        "xrs_encode": ([P, PP, I, Z], I),
        "xrs_reconst_one": ([P, PP, I, Z, I], I),
        "xrs_reconst": ([P, PP, I, Z, IP, I, IP, I], I),
        "xrs_update": ([P, P, P, Z, I, PP, I], I),
        "xrs_replace": ([P, PP, IP, I, Z, PP, I], I),
        "xrs_batch_strides": ([Z, I, ctypes.POINTER(Z), ctypes.POINTER(Z)], I),
        "xrs_batch_layout": ([Z, I, ctypes.POINTER(Z), ctypes.POINTER(Z), ctypes.POINTER(Z)], I),
        "xrs_encode_batched": ([P, P, Z, Z, Z, Z, P], I),
        "xrs_reconst_one_batched": ([P, P, Z, Z, Z, Z, I, P], I),
        "xrs_reconst_batched": ([P, P, Z, Z, Z, Z, IP, I, IP, I, P], I),
        "xrs_update_batched": ([P, P, Z, P, Z, Z, I, P, Z, Z, Z, P], I),
        "xrs_update_rows_batched": ([P, P, Z, P, Z, Z, P, P, Z, Z, Z, P], I),
        "xrs_replace_batched": ([P, P, Z, Z, IP, I, Z, P, Z, Z, Z, P], I),
        "xrs_encode_host": ([P, P, Z, Z, Z, Z], I),
        "xrs_reconst_one_host": ([P, P, Z, Z, Z, Z, I], I),
        "xrs_reconst_host": ([P, P, Z, Z, Z, Z, IP, I, IP, I], I),
        "xrs_update_host": ([P, P, Z, P, Z, Z, I, P, Z, Z, Z], I),
        "xrs_replace_host": ([P, P, Z, Z, IP, I, Z, P, Z, Z, Z], I),
        "xrs_host_alloc": ([Z], P),
        "xrs_host_free": ([P], None),
        "xrs_host_register": ([P, Z], I),
        "xrs_host_unregister": ([P], I),
        "xrs_host_device_pointer": ([P], P),
        "xrs_encode_shards": ([P, PP, Z, Z, Z, P], I),
        "xrs_reconst_one_shards": ([P, PP, Z, Z, Z, I, P], I),
        "xrs_reconst_shards": ([P, PP, Z, Z, Z, IP, I, IP, I, P], I),
        "xrs_enable_peer_access": ([I, I], I),
        "xrs_queue_new": ([P, Z, Z, I, ctypes.POINTER(P)], I),
        "xrs_queue_free": ([P], None),
        "xrs_queue_encode": ([P, PP, I], I),
        "xrs_queue_reconst_one": ([P, PP, I, I], I),
        "xrs_queue_update": ([P, P, P, I, PP, I], I),
        "xrs_queue_reconst": ([P, PP, I, IP, I, IP, I], I),
        "xrs_queue_replace": ([P, PP, IP, I, PP, I], I),
        "xrs_queue_submit_encode": ([P, PP, I, ctypes.POINTER(P)], I),
        "xrs_queue_submit_reconst_one": ([P, PP, I, I, ctypes.POINTER(P)], I),
        "xrs_queue_submit_update": ([P, P, P, I, PP, I, ctypes.POINTER(P)], I),
        "xrs_queue_submit_reconst": ([P, PP, I, IP, I, IP, I, ctypes.POINTER(P)], I),
        "xrs_queue_submit_replace": ([P, PP, IP, I, PP, I, ctypes.POINTER(P)], I),
        "xrs_queue_poll": ([P], I),
        "xrs_queue_wait": ([P], I),
        "xrs_queue_batch_stripes": ([P], Z),
        "xrs_queue_stats": ([P, ctypes.POINTER(ctypes.c_uint64)], I),
        "xrs_queue_batch_sizes": ([P, ctypes.POINTER(ctypes.c_uint64), I], I),
        "xrs_queue_dump": ([P, ctypes.c_char_p, Z], Z),
        "xrs_group_new": ([I, I, IP, I, ctypes.POINTER(P)], I),
        "xrs_group_free": ([P], None),
        "xrs_group_size": ([P], I),
        "xrs_group_codec": ([P, I], P),
        "xrs_group_encode_host": ([P, P, Z, Z, Z, Z], I),
        "xrs_group_reconst_one_host": ([P, P, Z, Z, Z, Z, I], I),
        "xrs_group_reconst_host": ([P, P, Z, Z, Z, Z, IP, I, IP, I], I),
        "xrs_group_update_host": ([P, P, Z, P, Z, Z, I, P, Z, Z, Z], I),
        "xrs_group_replace_host": ([P, P, Z, Z, IP, I, Z, P, Z, Z, Z], I),
    }
    for name, (args, res) in sig.items():
        try:
            f = getattr(L, name)
        except AttributeError:
            if os.environ.get("XRS_LIB"):  # an older build for A/B: its own symbol set
                continue
            raise
        f.argtypes = args
        f.restype = res
    return L


_lib = _load()


def lib():
    return _lib


def _ptr(buf) -> int:
    """Address of a writable host buffer (numpy array, bytearray, ctypes array)."""
    if hasattr(buf, "ctypes"):
        return buf.ctypes.data
    if isinstance(buf, bytearray):
        return ctypes.addressof((ctypes.c_char * len(buf)).from_buffer(buf))
    return ctypes.addressof(buf)


def _nbytes(buf) -> int:
    if hasattr(buf, "nbytes"):
        return int(buf.nbytes)
    if isinstance(buf, (bytearray, bytes)):
        return len(buf)
    return ctypes.sizeof(buf)


def _check_lens(size: int, *groups, exact: bool = False) -> None:
    """Every (non-None) vect in `groups` is `size` bytes: the C ABI reads and
    writes `size` bytes of each, so a shorter one would be overrun.  Checked
    after the even-size rule (xrs.go:105 checkSize runs first) unless `exact`
    (a queue's fixed size)."""
    if size & 1 and not exact:
        return
    for g in groups:
        for v in g:
            if v is not None and _nbytes(v) != size:
                raise XRSError(XRS_ERR_ILLEGAL_VECTS, "illegal vects")


def _ptrs(vects):
    a = (ctypes.c_void_p * max(1, len(vects)))()
    for i, v in enumerate(vects):
        a[i] = None if v is None else _ptr(v)
    return a


def _ints(xs):
    a = (ctypes.c_int * max(1, len(xs)))()
    for i, v in enumerate(xs):
        a[i] = int(v)
    return a


def batch_strides(size: int, n_shards: int):
    """Recommended (shard_stride, stripe_stride) for a device batch."""
    a, b = ctypes.c_size_t(), ctypes.c_size_t()
    _raise(_lib.xrs_batch_strides(size, n_shards, ctypes.byref(a), ctypes.byref(b)))
    return a.value, b.value


def batch_layout(size: int, n_shards: int):
    """Recommended (shard_stride, stripe_stride, base_offset) for a device
    batch: place it at a 16-B-aligned address + base_offset (odd vect sizes
    get their b-halves aligned; xrs_batch_layout)."""
    a, b, c = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    _raise(_lib.xrs_batch_layout(size, n_shards, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
    return a.value, b.value, c.value


def source_hash(root: str | None = None) -> str:
    """The digest the Makefile embeds in xrs_version() (xrs_amd/csrc/version.cpp),
    computed from the source tree at `root` (default: this checkout): sha256 of
    xrs_amd/csrc's Makefile and *.cpp *.h *.hip *.map in byte order of their
    names, then include/xrs_hip.h; first 16 hex digits."""
    import glob
    import hashlib

    root = root or os.path.dirname(_HERE)
    csrc = os.path.join(root, "xrs_amd", "csrc")
    names = {os.path.basename(f) for pat in ("*.cpp", "*.h", "*.hip", "*.map")
             for f in glob.glob(os.path.join(csrc, pat))} | {"Makefile"}
    files = [os.path.join(csrc, n) for n in sorted(names, key=lambda n: n.encode())]
    files.append(os.path.join(root, "include", "xrs_hip.h"))
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def version() -> str:
    """xrs_version(): "xrs-hip <v> gfx950 src <source digest>"."""
    return _lib.xrs_version().decode()


def library_source_hash() -> str:
    """The source digest the loaded library was built with (see source_hash)."""
    v = version().split()
    return v[v.index("src") + 1] if "src" in v else "unknown"


def trace_kernels(on: bool = True) -> None:
    """Start (clearing the record) or stop recording the kernels the library
    launches (xrs_trace_kernels; diagnostics)."""
    _lib.xrs_trace_kernels(1 if on else 0)


def traced_kernels() -> dict:
    """{kernel instantiation: launches} recorded since trace_kernels(True)."""
    n = _lib.xrs_traced_kernels(None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    _lib.xrs_traced_kernels(buf, n + 1)
    out = {}
    for ln in buf.value.decode().splitlines():
        name, _, cnt = ln.rpartition(" ")
        out[name] = int(cnt)
    return out


def _raise(code: int, arg: int = 0):
    if code == 0:
        return
    buf = ctypes.create_string_buffer(128)
    _lib.xrs_format_error(code, int(arg), buf, len(buf))
    raise XRSError(code, buf.value.decode())


class XRS:
    """The X-Reed-Solomon codec (mirror of Go ``type XRS``, xrs.go:42-50)."""

    def __init__(self, data_num: int, parity_num: int):
        h = ctypes.c_void_p()
        _raise(_lib.xrs_new(int(data_num), int(parity_num), ctypes.byref(h)))
        self._h = h
        self.data_num = _lib.xrs_data_num(h)
        self.parity_num = _lib.xrs_parity_num(h)

    def __del__(self, _free=_lib.xrs_free):  # bound now: module globals are gone at exit
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _free(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    # ---------------------------------------------------------- codec state
    @property
    def gen_matrix(self) -> bytes:
        n = (self.data_num + self.parity_num) * self.data_num
        buf = ctypes.create_string_buffer(n)
        _raise(_lib.xrs_gen_matrix(self._h, buf, n))
        return buf.raw

    @property
    def xor_set(self) -> dict:
        """x.XORSet (xrs.go:49): parity index -> data indexes."""
        out = {}
        cap = self.data_num
        arr = (ctypes.c_int * max(1, cap))()
        n = ctypes.c_int()
        for h in range(self.data_num + 1, self.data_num + self.parity_num):
            _raise(_lib.xrs_xorset(self._h, h, arr, cap, ctypes.byref(n)))
            if n.value:
                out[h] = [arr[i] for i in range(n.value)]
        return out

    def get_need_vects(self, need_reconst: int):
        """xrs.go:146 GetNeedVects -> (aNeed, bNeed)."""
        a = (ctypes.c_int * max(1, self.data_num))()
        n = ctypes.c_int()
        b = (ctypes.c_int * 2)()
        _raise(_lib.xrs_get_need_vects(self._h, int(need_reconst), a, ctypes.byref(n), b),
               need_reconst)
        return [a[i] for i in range(n.value)], [b[0], b[1]]

    # ------------------------------------------------------- sync (host) API
    def encode(self, vects) -> None:
        size = _nbytes(vects[0]) if len(vects) else 0
        _check_lens(size, vects)
        _raise(_lib.xrs_encode(self._h, _ptrs(vects), len(vects), size), size)

    def reconst_one(self, vects, need_reconst: int) -> None:
        size = _nbytes(vects[0])
        _check_lens(size, vects)
        rc = _lib.xrs_reconst_one(self._h, _ptrs(vects), len(vects), size, int(need_reconst))
        _raise(rc, size if rc == XRS_ERR_SIZE_NOT_EVEN else need_reconst)

    def reconst(self, vects, dp_has, need_reconst) -> None:
        size = _nbytes(vects[0])
        _check_lens(size, vects)
        rc = _lib.xrs_reconst(self._h, _ptrs(vects), len(vects), size, _ints(dp_has),
                              len(dp_has), _ints(need_reconst), len(need_reconst))
        arg = size if rc == XRS_ERR_SIZE_NOT_EVEN else (need_reconst[0] if need_reconst else 0)
        _raise(rc, arg)

    def update(self, old_data, new_data, row: int, parity) -> None:
        size = _nbytes(old_data)
        _check_lens(size, [new_data], parity)
        rc = _lib.xrs_update(self._h, _ptr(old_data), _ptr(new_data), size, int(row),
                             _ptrs(parity), len(parity))
        _raise(rc, size if rc == XRS_ERR_SIZE_NOT_EVEN else row)

    def replace(self, data, replace_rows, parity) -> None:
        size = _nbytes(data[0]) if len(data) else 0
        _check_lens(size, data, parity)
        rc = _lib.xrs_replace(self._h, _ptrs(data), _ints(replace_rows), len(replace_rows), size,
                              _ptrs(parity), len(parity))
        bad = next((r for r in replace_rows if r < 0 or r >= self.data_num), 0)
        _raise(rc, size if rc == XRS_ERR_SIZE_NOT_EVEN else bad)

    # ------------------------------------------- per-shard pointer tables
    # shards: list of d+p device addresses (int); stripe s of shard i at
    # shards[i] + s*stripe_stride.  Shards may live on peer GPUs (xGMI).
    def encode_shards(self, shards, stripe_stride: int, size: int, n_stripes: int,
                      stream: int = 0) -> None:
        t = (ctypes.c_void_p * len(shards))(*shards)
        _raise(_lib.xrs_encode_shards(self._h, t, stripe_stride, size, n_stripes, stream), size)

    def reconst_one_shards(self, shards, stripe_stride: int, size: int, n_stripes: int, k: int,
                           stream: int = 0) -> None:
        t = (ctypes.c_void_p * len(shards))(*[s or 0 for s in shards])
        rc = _lib.xrs_reconst_one_shards(self._h, t, stripe_stride, size, n_stripes, int(k), stream)
        _raise(rc, size if rc == XRS_ERR_SIZE_NOT_EVEN else k)

    def reconst_shards(self, shards, stripe_stride: int, size: int, n_stripes: int, dp_has,
                       need_reconst, stream: int = 0) -> None:
        t = (ctypes.c_void_p * len(shards))(*shards)
        rc = _lib.xrs_reconst_shards(self._h, t, stripe_stride, size, n_stripes, _ints(dp_has),
                                     len(dp_has), _ints(need_reconst), len(need_reconst), stream)
        arg = size if rc == XRS_ERR_SIZE_NOT_EVEN else (need_reconst[0] if need_reconst else 0)
        _raise(rc, arg)

    # ------------------------------------------- host-resident pipelined API
    # host_base: address of a host buffer (pinned for full PCIe rate).
    def encode_host(self, host_base: int, size: int, shard_stride: int, stripe_stride: int,
                    n_stripes: int) -> None:
        _raise(_lib.xrs_encode_host(self._h, host_base, size, shard_stride, stripe_stride,
                                    n_stripes), size)

    def reconst_one_host(self, host_base: int, size: int, shard_stride: int, stripe_stride: int,
                         n_stripes: int, k: int) -> None:
        rc = _lib.xrs_reconst_one_host(self._h, host_base, size, shard_stride, stripe_stride,
                                       n_stripes, int(k))
        _raise(rc, size if rc == XRS_ERR_SIZE_NOT_EVEN else k)

    def reconst_host(self, host_base: int, size: int, shard_stride: int, stripe_stride: int,
                     n_stripes: int, dp_has, need_reconst) -> None:
        rc = _lib.xrs_reconst_host(self._h, host_base, size, shard_stride, stripe_stride,
                                   n_stripes, _ints(dp_has), len(dp_has), _ints(need_reconst),
                                   len(need_reconst))
        arg = size if rc == XRS_ERR_SIZE_NOT_EVEN else (need_reconst[0] if need_reconst else 0)
        _raise(rc, arg)

    def update_host(self, old_base: int, old_stripe_stride: int, new_base: int,
                    new_stripe_stride: int, size: int, row: int, parity_base: int,
                    parity_shard_stride: int, parity_stripe_stride: int, n_stripes: int) -> None:
        rc = _lib.xrs_update_host(self._h, old_base, old_stripe_stride, new_base,
                                  new_stripe_stride, size, int(row), parity_base,
                                  parity_shard_stride, parity_stripe_stride, n_stripes)
        _raise(rc, size if rc == XRS_ERR_SIZE_NOT_EVEN else row)

    def replace_host(self, data_base: int, data_shard_stride: int, data_stripe_stride: int,
                     replace_rows, size: int, parity_base: int, parity_shard_stride: int,
                     parity_stripe_stride: int, n_stripes: int) -> None:
        rc = _lib.xrs_replace_host(self._h, data_base, data_shard_stride, data_stripe_stride,
                                   _ints(replace_rows), len(replace_rows), size, parity_base,
                                   parity_shard_stride, parity_stripe_stride, n_stripes)
        bad = next((r for r in replace_rows if r < 0 or r >= self.data_num), 0)
        _raise(rc, size if rc == XRS_ERR_SIZE_NOT_EVEN else bad)

    # ------------------------------------------- batched device-resident API
    # Pointers are device addresses (int); stream is a hipStream_t as int (0 = null).
    def encode_batched(self, base: int, size: int, shard_stride: int, stripe_stride: int,
                       n_stripes: int, stream: int = 0) -> None:
        _raise(_lib.xrs_encode_batched(self._h, base, size, shard_stride, stripe_stride,
                                       n_stripes, stream), size)

    def reconst_one_batched(self, base: int, size: int, shard_stride: int, stripe_stride: int,
                            n_stripes: int, k: int, stream: int = 0) -> None:
        rc = _lib.xrs_reconst_one_batched(self._h, base, size, shard_stride, stripe_stride,
                                          n_stripes, int(k), stream)
        _raise(rc, size if rc == XRS_ERR_SIZE_NOT_EVEN else k)

    def reconst_batched(self, base: int, size: int, shard_stride: int, stripe_stride: int,
                        n_stripes: int, dp_has, need_reconst, stream: int = 0) -> None:
        rc = _lib.xrs_reconst_batched(self._h, base, size, shard_stride, stripe_stride, n_stripes,
                                      _ints(dp_has), len(dp_has), _ints(need_reconst),
                                      len(need_reconst), stream)
        arg = size if rc == XRS_ERR_SIZE_NOT_EVEN else (need_reconst[0] if need_reconst else 0)
        _raise(rc, arg)

    def update_batched(self, old_base: int, old_stripe_stride: int, new_base: int,
                       new_stripe_stride: int, size: int, row: int, parity_base: int,
                       parity_shard_stride: int, parity_stripe_stride: int, n_stripes: int,
                       stream: int = 0) -> None:
        rc = _lib.xrs_update_batched(self._h, old_base, old_stripe_stride, new_base,
                                     new_stripe_stride, size, int(row), parity_base,
                                     parity_shard_stride, parity_stripe_stride, n_stripes, stream)
        _raise(rc, size if rc == XRS_ERR_SIZE_NOT_EVEN else row)

    def update_rows_batched(self, old_base: int, old_stripe_stride: int, new_base: int,
                            new_stripe_stride: int, size: int, rows_base: int, parity_base: int,
                            parity_shard_stride: int, parity_stripe_stride: int, n_stripes: int,
                            stream: int = 0) -> None:
        """Update with one data row per stripe; rows_base: device-readable
        address of n_stripes int32 rows (rows outside [0, d) are skipped)."""
        _raise(_lib.xrs_update_rows_batched(self._h, old_base, old_stripe_stride, new_base,
                                            new_stripe_stride, size, rows_base, parity_base,
                                            parity_shard_stride, parity_stripe_stride, n_stripes,
                                            stream), size)

    def replace_batched(self, data_base: int, data_shard_stride: int, data_stripe_stride: int,
                        replace_rows, size: int, parity_base: int, parity_shard_stride: int,
                        parity_stripe_stride: int, n_stripes: int, stream: int = 0) -> None:
        rc = _lib.xrs_replace_batched(self._h, data_base, data_shard_stride, data_stripe_stride,
                                      _ints(replace_rows), len(replace_rows), size, parity_base,
                                      parity_shard_stride, parity_stripe_stride, n_stripes, stream)
        bad = next((r for r in replace_rows if r < 0 or r >= self.data_num), 0)
        _raise(rc, size if rc == XRS_ERR_SIZE_NOT_EVEN else bad)


class XRSGroup:
    """One process driving several GPUs (xrs_group_*): one codec per listed
    device; host-resident batches are split into contiguous stripe ranges and
    run concurrently, each GPU over its own PCIe link."""

    def __init__(self, data_num: int, parity_num: int, devices):
        devs = [int(d) for d in devices]
        h = ctypes.c_void_p()
        _raise(_lib.xrs_group_new(int(data_num), int(parity_num), _ints(devs), len(devs),
                                  ctypes.byref(h)))
        self._h = h
        self.devices = devs
        self.data_num = int(data_num)

    def __del__(self, _free=_lib.xrs_group_free):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _free(h)
            self._h = None

    def __len__(self) -> int:
        return _lib.xrs_group_size(self._h)

    def encode_host(self, host_base: int, size: int, shard_stride: int, stripe_stride: int,
                    n_stripes: int) -> None:
        _raise(_lib.xrs_group_encode_host(self._h, host_base, size, shard_stride, stripe_stride,
                                          n_stripes), size)

    def reconst_one_host(self, host_base: int, size: int, shard_stride: int, stripe_stride: int,
                         n_stripes: int, need_reconst: int) -> None:
        rc = _lib.xrs_group_reconst_one_host(self._h, host_base, size, shard_stride,
                                             stripe_stride, n_stripes, int(need_reconst))
        _raise(rc, size if rc == XRS_ERR_SIZE_NOT_EVEN else need_reconst)

    def update_host(self, old_base: int, old_stripe_stride: int, new_base: int,
                    new_stripe_stride: int, size: int, row: int, parity_base: int,
                    parity_shard_stride: int, parity_stripe_stride: int, n_stripes: int) -> None:
        rc = _lib.xrs_group_update_host(self._h, old_base, old_stripe_stride, new_base,
                                        new_stripe_stride, size, int(row), parity_base,
                                        parity_shard_stride, parity_stripe_stride, n_stripes)
        _raise(rc, size if rc == XRS_ERR_SIZE_NOT_EVEN else row)

    def replace_host(self, data_base: int, data_shard_stride: int, data_stripe_stride: int,
                     replace_rows, size: int, parity_base: int, parity_shard_stride: int,
                     parity_stripe_stride: int, n_stripes: int) -> None:
        rc = _lib.xrs_group_replace_host(self._h, data_base, data_shard_stride,
                                         data_stripe_stride, _ints(replace_rows),
                                         len(replace_rows), size, parity_base,
                                         parity_shard_stride, parity_stripe_stride, n_stripes)
        bad = next((r for r in replace_rows if r < 0 or r >= self.data_num), 0)
        _raise(rc, size if rc == XRS_ERR_SIZE_NOT_EVEN else bad)

    def reconst_host(self, host_base: int, size: int, shard_stride: int, stripe_stride: int,
                     n_stripes: int, dp_has, need_reconst) -> None:
        rc = _lib.xrs_group_reconst_host(self._h, host_base, size, shard_stride, stripe_stride,
                                         n_stripes, _ints(dp_has), len(dp_has),
                                         _ints(need_reconst), len(need_reconst))
        arg = size if rc == XRS_ERR_SIZE_NOT_EVEN else (need_reconst[0] if need_reconst else 0)
        _raise(rc, arg)


class XRSQueue:
    """Batching queue over a codec (xrs_queue_*): per-stripe Encode /
    ReconstOne calls from many threads are coalesced into device batches.
    ctypes releases the GIL during each call, so Python threads batch too."""

    def __init__(self, codec: XRS, size: int, max_batch_stripes: int = 1024,
                 max_wait_us: int = 50):
        self._h = None
        self._cv = threading.Condition()
        self._inflight = 0
        h = ctypes.c_void_p()
        _raise(_lib.xrs_queue_new(codec.handle, size, max_batch_stripes, max_wait_us,
                                  ctypes.byref(h)), size)
        self._codec = codec  # keep the codec alive
        self._h = h
        self.size = size
        self.batch_stripes = _lib.xrs_queue_batch_stripes(h)

    @property
    def handle(self):
        """The xrs_queue* (for callers that drive the C ABI directly)."""
        return self._h

    def close(self, _free=_lib.xrs_queue_free):
        """New calls fail from here on; calls in flight complete first."""
        with self._cv:
            h, self._h = self._h, None
            self._cv.wait_for(lambda: self._inflight == 0)
        if h is not None and h.value:
            _free(h)

    def __del__(self):
        self.close()

    def _call(self, fn, *args):
        with self._cv:
            h = self._h
            if h is None:
                return XRS_ERR_INVALID_ARG
            self._inflight += 1
        try:
            return fn(h, *args)
        finally:
            with self._cv:
                self._inflight -= 1
                self._cv.notify_all()

    def encode(self, vects) -> None:
        _check_lens(self.size, vects, exact=True)
        _raise(self._call(_lib.xrs_queue_encode, _ptrs(vects), len(vects)), self.size)

    def reconst_one(self, vects, need_reconst: int) -> None:
        _check_lens(self.size, vects, exact=True)
        _raise(self._call(_lib.xrs_queue_reconst_one, _ptrs(vects), len(vects),
                          int(need_reconst)), need_reconst)

    def reconst(self, vects, dp_has, need_reconst) -> None:
        _check_lens(self.size, vects, exact=True)
        rc = self._call(_lib.xrs_queue_reconst, _ptrs(vects), len(vects), _ints(dp_has),
                        len(dp_has), _ints(need_reconst), len(need_reconst))
        arg = self.size if rc == XRS_ERR_SIZE_NOT_EVEN else (need_reconst[0] if need_reconst else 0)
        _raise(rc, arg)

    def replace(self, data, replace_rows, parity) -> None:
        _check_lens(self.size, data, parity, exact=True)
        rc = self._call(_lib.xrs_queue_replace, _ptrs(data), _ints(replace_rows),
                        len(replace_rows), _ptrs(parity), len(parity))
        bad = next((r for r in replace_rows if r < 0 or r >= self._codec.data_num), 0)
        _raise(rc, bad)

    def update(self, old_data, new_data, row: int, parity) -> None:
        _check_lens(self.size, [old_data, new_data], parity, exact=True)
        _raise(self._call(_lib.xrs_queue_update, _ptr(old_data), _ptr(new_data), int(row),
                          _ptrs(parity), len(parity)), row)

    # ---- asynchronous forms (xrs_queue_submit_* / xrs_queue_wait) ----------
    def _submit(self, fn, keep, arg, *args):
        """Stage one call; a QueueTicket, or None when no staging batch is
        free (XRS_ERR_BUSY: nothing staged, wait on a ticket and resubmit)."""
        with self._cv:
            h = self._h
            if h is None:
                _raise(XRS_ERR_INVALID_ARG)
            self._inflight += 1  # until the ticket is waited on (close() waits)
        t = ctypes.c_void_p()
        rc = fn(h, *args, ctypes.byref(t))
        if rc != 0:
            self._done()
            if rc == XRS_ERR_BUSY:
                return None
            _raise(rc, arg)
        return QueueTicket(self, t, keep, arg)

    def _done(self):
        with self._cv:
            self._inflight -= 1
            self._cv.notify_all()

    def submit_encode(self, vects):
        _check_lens(self.size, vects, exact=True)
        return self._submit(_lib.xrs_queue_submit_encode, vects, self.size, _ptrs(vects), len(vects))

    def submit_reconst_one(self, vects, need_reconst: int):
        _check_lens(self.size, vects, exact=True)
        return self._submit(_lib.xrs_queue_submit_reconst_one, vects, need_reconst, _ptrs(vects),
                            len(vects), int(need_reconst))

    def submit_reconst(self, vects, dp_has, need_reconst):
        _check_lens(self.size, vects, exact=True)
        arg = need_reconst[0] if need_reconst else 0
        return self._submit(_lib.xrs_queue_submit_reconst, vects, arg, _ptrs(vects), len(vects),
                            _ints(dp_has), len(dp_has), _ints(need_reconst), len(need_reconst))

    def submit_replace(self, data, replace_rows, parity):
        _check_lens(self.size, data, parity, exact=True)
        bad = next((r for r in replace_rows if r < 0 or r >= self._codec.data_num), 0)
        return self._submit(_lib.xrs_queue_submit_replace, (data, parity), bad, _ptrs(data),
                            _ints(replace_rows), len(replace_rows), _ptrs(parity), len(parity))

    def submit_update(self, old_data, new_data, row: int, parity):
        _check_lens(self.size, [old_data, new_data], parity, exact=True)
        return self._submit(_lib.xrs_queue_submit_update, (old_data, new_data, parity), row,
                            _ptr(old_data), _ptr(new_data), int(row), _ptrs(parity), len(parity))

    def stats(self) -> dict:
        """Batches and stripes run so far, and summed device / queueing ns."""
        out = (ctypes.c_uint64 * 4)()
        _raise(_lib.xrs_queue_stats(self._h, out))
        return {"batches": out[0], "stripes": out[1], "run_ns": out[2], "wait_ns": out[3]}

    def batch_sizes(self) -> dict:
        """{stripes per batch: batches run} since the queue was made
        (xrs_queue_batch_sizes; counts past 64 stripes are kept as 64)."""
        out = (ctypes.c_uint64 * 65)()
        _raise(_lib.xrs_queue_batch_sizes(self._h, out, 65))
        return {n: int(c) for n, c in enumerate(out) if c}

    def dump(self) -> str:
        """The queue's state as text (xrs_queue_dump): per staging batch its
        state, reserved / staged / released slots, launches and completion word."""
        n = _lib.xrs_queue_dump(self._h, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        _lib.xrs_queue_dump(self._h, buf, n + 1)
        return buf.value.decode()


class QueueTicket:
    """One staged asynchronous call (XRSQueue.submit_*): wait() blocks until
    its stripe is done, copies the outputs back and raises the call's error;
    done() polls.  Holds the call's buffers until waited on; every ticket is
    waited on once (an abandoned ticket is waited on when collected)."""

    def __init__(self, q: XRSQueue, handle, keep, arg):
        self._q, self._t, self._keep, self._arg = q, handle, keep, arg

    def done(self) -> bool:
        return self._t is None or _lib.xrs_queue_poll(self._t) == 1

    def wait(self) -> None:
        t, self._t = self._t, None
        if t is None:
            return
        try:
            rc = _lib.xrs_queue_wait(t)
        finally:
            self._keep = None
            self._q._done()
        _raise(rc, self._arg)

    def __del__(self):
        if self._t is not None:
            try:
                self.wait()
            except XRSError:
                pass
