"""ctypes binding of oracle/build/libxrs_oracle.so -- TEST INFRASTRUCTURE ONLY.

Used by tests/ (cross-check of the two CPU restatements and of the GPU path)
and by bench.py's cpu_baseline leg.  The product package never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libxrs_oracle.so")
_lib = None

ERRORS = {
    -1: "illegal parity",
    -2: "vect size not even",
    -3: "illegal data index",
    -4: "illegal vects",
    -5: "too few survivors",
    -6: "illegal index",
    -7: "singular matrix",
}


class OracleError(Exception):
    def __init__(self, code: int):
        super().__init__(f"{ERRORS.get(code, 'error')} ({code})")
        self.code = code


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        I = ctypes.c_int
        Z = ctypes.c_size_t
        IP = ctypes.POINTER(ctypes.c_int)
        PP = ctypes.POINTER(ctypes.c_void_p)
        L.oxrs_sizeof.restype = Z
        L.oxrs_new.argtypes = [I, I, P]
        L.oxrs_gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.oxrs_gf_mul.restype = ctypes.c_uint8
        L.oxrs_get_need_vects.argtypes = [P, I, IP, IP, IP]
        L.oxrs_encode.argtypes = [P, PP, I, Z]
        L.oxrs_reconst_one.argtypes = [P, PP, I, Z, I]
        L.oxrs_reconst.argtypes = [P, PP, I, Z, IP, I, IP, I]
        L.oxrs_retrieve_rs.argtypes = [P, PP, I, Z, IP, I]
        L.oxrs_update.argtypes = [P, P, P, Z, I, PP]
        L.oxrs_replace.argtypes = [P, PP, IP, I, Z, PP]
        L.oxrs_encode_batch.argtypes = [P, P, Z, Z, ctypes.c_long, I]
        L.oxrs_reconst_one_batch.argtypes = [P, P, Z, Z, ctypes.c_long, I, I]
        L.oxrs_update_batch.argtypes = [P, P, Z, Z, ctypes.c_long, I, I]
        L.oxrs_replace_batch.argtypes = [P, P, Z, Z, ctypes.c_long, IP, I, I]
        L.oxrs_simd_available.restype = I
        L.oxrs_simd_level.restype = I
        _lib = L
    return _lib


def _ptrs(arrs):
    a = (ctypes.c_void_p * max(1, len(arrs)))()
    for i, v in enumerate(arrs):
        a[i] = v.ctypes.data
    return a


def _ints(xs):
    a = (ctypes.c_int * max(1, len(xs)))()
    for i, v in enumerate(xs):
        a[i] = int(v)
    return a


def _chk(rc):
    if rc != 0:
        raise OracleError(rc)


class OracleXRS:
    """The C restatement behind the same method names as oracle.xrs_oracle.XRS."""

    def __init__(self, d: int, p: int):
        L = lib()
        self._buf = ctypes.create_string_buffer(L.oxrs_sizeof())
        _chk(L.oxrs_new(d, p, self._buf))
        self.d, self.p = d, p

    @property
    def handle(self):
        return self._buf

    def get_need_vects(self, k):
        a = (ctypes.c_int * 256)()
        n = ctypes.c_int()
        b = (ctypes.c_int * 2)()
        _chk(lib().oxrs_get_need_vects(self._buf, k, a, ctypes.byref(n), b))
        return [a[i] for i in range(n.value)], [b[0], b[1]]

    def encode(self, vects):
        _chk(lib().oxrs_encode(self._buf, _ptrs(vects), len(vects), len(vects[0])))

    def reconst_one(self, vects, k):
        _chk(lib().oxrs_reconst_one(self._buf, _ptrs(vects), len(vects), len(vects[0]), k))

    def reconst(self, vects, dp_has, need):
        _chk(lib().oxrs_reconst(self._buf, _ptrs(vects), len(vects), len(vects[0]),
                                _ints(dp_has), len(dp_has), _ints(need), len(need)))

    def retrieve_rs(self, vects, dp_has):
        _chk(lib().oxrs_retrieve_rs(self._buf, _ptrs(vects), len(vects), len(vects[0]),
                                    _ints(dp_has), len(dp_has)))

    def update(self, old, new, row, parity):
        _chk(lib().oxrs_update(self._buf, old.ctypes.data, new.ctypes.data, len(old), row,
                               _ptrs(parity)))

    def replace(self, data, rows, parity):
        _chk(lib().oxrs_replace(self._buf, _ptrs(data), _ints(rows), len(rows), len(data[0]),
                                _ptrs(parity)))

    # ---- CPU baseline over a contiguous batch [n_stripes][d+p][size]
    def encode_batch(self, buf: np.ndarray, size: int, n_stripes: int, threads: int = 1):
        _chk(lib().oxrs_encode_batch(self._buf, buf.ctypes.data, size,
                                     (self.d + self.p) * size, n_stripes, threads))

    def reconst_one_batch(self, buf: np.ndarray, size: int, n_stripes: int, k: int,
                          threads: int = 1):
        _chk(lib().oxrs_reconst_one_batch(self._buf, buf.ctypes.data, size,
                                          (self.d + self.p) * size, n_stripes, k, threads))

    def update_batch(self, buf: np.ndarray, size: int, n_stripes: int, row: int,
                     threads: int = 1):
        """buf: [n_stripes][2 + p][size] = old, new, parity (parity updated)."""
        _chk(lib().oxrs_update_batch(self._buf, buf.ctypes.data, size, (2 + self.p) * size,
                                     n_stripes, row, threads))

    def replace_batch(self, buf: np.ndarray, size: int, n_stripes: int, rows, threads: int = 1):
        """buf: [n_stripes][len(rows) + p][size] = data, parity (parity updated)."""
        _chk(lib().oxrs_replace_batch(self._buf, buf.ctypes.data, size,
                                      (len(rows) + self.p) * size, n_stripes, _ints(rows),
                                      len(rows), threads))
