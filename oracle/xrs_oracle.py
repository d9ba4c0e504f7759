"""Independent numpy restatement of templexxx/xrs -- TEST INFRASTRUCTURE ONLY.

This module and ``oracle/xrs_oracle.c`` are the parity checkers for the HIP
product path.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg import anything under ``oracle/``; the product package
``xrs_amd`` never does.

It is deliberately written separately from the C restatement (own GF tables,
own matrix inverse, own control flow) so the two cross-check each other; both
are pinned to the reference's only known-answer test, TestXRS_Encode
(/root/reference/xrs_test.go:102-122).

Reference citations (file:line under /root/reference):
  New            xrs.go:55-68      makeXORSet   xrs.go:77-100
  Encode         xrs.go:103-128    checkSize    xrs.go:130-136
  GetNeedVects   xrs.go:146-171    ReconstOne   xrs.go:175-221
  Reconst        xrs.go:236-301    retrieveRS   xrs.go:305-320
  Update         xrs.go:324-346    Replace      xrs.go:363-387
The RS arithmetic is the un-vendored dependency github.com/templexxx/
reedsolomon v1.1.3 (go.mod:6): GF(2^8)/0x11d, identity + Cauchy inv(i^j).
"""
from __future__ import annotations

import numpy as np

POLY = 0x11D


class XRSError(Exception):
    """Error carrying the reference's message text (xrs.go) or a [dep] one."""


def _tables():
    exp = np.zeros(512, dtype=np.uint8)
    log = np.zeros(256, dtype=np.int32)
    v = 1
    for i in range(255):
        exp[i] = v
        log[v] = i
        v <<= 1
        if v & 0x100:
            v ^= POLY
    exp[255:510] = exp[0:255]
    return exp, log


EXP, LOG = _tables()
# full 256x256 product table (64 KiB): MUL[a, b] = a*b in GF(2^8)
MUL = np.zeros((256, 256), dtype=np.uint8)
for _a in range(1, 256):
    MUL[_a, 1:] = EXP[LOG[_a] + LOG[np.arange(1, 256)]]
del _a


def gf_mul(a: int, b: int) -> int:
    return int(MUL[a, b])


def gf_inv(a: int) -> int:
    if a == 0:
        raise ZeroDivisionError("inverse of 0 in GF(2^8)")
    return int(EXP[255 - LOG[a]])


def gf_mat_inv(m: np.ndarray) -> np.ndarray:
    """Gauss-Jordan inverse over GF(2^8); raises XRSError if singular."""
    n = m.shape[0]
    a = np.concatenate([m.astype(np.uint8), np.eye(n, dtype=np.uint8)], axis=1)
    for c in range(n):
        piv = next((r for r in range(c, n) if a[r, c]), None)
        if piv is None:
            raise XRSError("matrix is singular")
        if piv != c:
            a[[c, piv]] = a[[piv, c]]
        a[c] = MUL[gf_inv(int(a[c, c])), a[c]]
        for r in range(n):
            if r != c and a[r, c]:
                a[r] ^= MUL[int(a[r, c]), a[c]]
    return a[:, n:].copy()


def gf_vec_mul(c: int, v: np.ndarray) -> np.ndarray:
    return MUL[c][v]


class XRS:
    """Mirror of the Go ``*XRS`` method set, over numpy uint8 arrays (in place)."""

    def __init__(self, data_num: int, parity_num: int):
        # xrs.go:56-59
        if parity_num == 1:
            raise XRSError("illegal parity")
        # reedsolomon.New validity [dep]; xrs_test.go:125-134 needs d+p<=256 to work
        if data_num <= 0 or parity_num <= 0 or data_num + parity_num > 256:
            raise XRSError("illegal data/parity number")
        self.d, self.p = data_num, parity_num
        d, p = data_num, parity_num
        g = np.zeros((d + p, d), dtype=np.uint8)
        g[:d] = np.eye(d, dtype=np.uint8)
        for i in range(d, d + p):
            for j in range(d):
                g[i, j] = gf_inv(i ^ j)
        self.gen = g
        self.xor_set = make_xor_set(d, p)

    # ---------------------------------------------------------------- helpers
    @staticmethod
    def _check_size(v) -> None:  # xrs.go:130-136
        if len(v) & 1:
            raise XRSError(f"vect size not even: {len(v)}")

    def get_need_vects(self, k: int):  # xrs.go:146-171
        d = self.d
        if k < 0 or k >= d:
            raise XRSError(f"illegal data index: {k}")
        b_need = [d, 0]
        for i, s in self.xor_set.items():
            if k in s:
                b_need[1] = i
                break
        a_need = [i for i in self.xor_set[b_need[1]] if i != k]
        return a_need, b_need

    # -------------------------------------------------------------- RS [dep]
    def rs_encode(self, vects) -> None:
        d, p = self.d, self.p
        if len(vects) != d + p:
            raise XRSError("illegal vects number")
        for r in range(p):
            acc = np.zeros(len(vects[0]), dtype=np.uint8)
            for j in range(d):
                acc ^= MUL[int(self.gen[d + r, j])][vects[j]]
            vects[d + r][:] = acc

    def rs_reconst(self, vects, dp_has, need) -> None:
        d, n = self.d, self.d + self.p
        if len(need) == 0:
            return
        if len(dp_has) < d:
            raise XRSError("too few survivors")
        if any(h < 0 or h >= n for h in dp_has) or any(t < 0 or t >= n for t in need):
            raise XRSError("illegal index")
        has = list(dp_has[:d])
        einv = gf_mat_inv(self.gen[has])
        outs = []
        for t in need:
            row = np.zeros(d, dtype=np.uint8)
            for j in range(d):  # gen[t] * Einv
                if self.gen[t, j]:
                    row ^= MUL[int(self.gen[t, j])][einv[j]]
            acc = np.zeros(len(vects[has[0]]), dtype=np.uint8)
            for i, h in enumerate(has):
                acc ^= MUL[int(row[i])][vects[h]]
            outs.append(acc)
        for t, o in zip(need, outs):
            vects[t][:] = o

    # ---------------------------------------------------------------- XRS API
    def encode(self, vects) -> None:  # xrs.go:103-128
        self._check_size(vects[0])
        self.rs_encode(vects)
        half = len(vects[0]) // 2
        for bi, xs in self.xor_set.items():
            for ai in xs:
                vects[bi][half:] ^= vects[ai][:half]

    def reconst_one(self, vects, k: int) -> None:  # xrs.go:175-221
        self._check_size(vects[0])
        a_need, b_need = self.get_need_vects(k)
        if len(vects) != self.d + self.p:
            raise XRSError("illegal vects number")
        half = len(vects[0]) // 2
        b_vects = [v[half:] for v in vects]
        d = self.d
        has = list(range(d))
        has[k] = d
        bi = b_need[1]
        b_rs = np.zeros(half, dtype=np.uint8)
        b_vects[bi] = b_rs
        self.rs_reconst(b_vects, has, [k, bi])
        a = vects[bi][half:] ^ b_rs
        for ai in a_need:
            a ^= vects[ai][:half]
        vects[k][:half] = a

    def retrieve_rs(self, vects, dp_has) -> None:  # xrs.go:305-320
        half = len(vects[0]) // 2
        for h in dp_has:
            if h > self.d:
                for ai in self.xor_set.get(h, []):
                    vects[h][half:] ^= vects[ai][:half]

    def reconst(self, vects, dp_has, need) -> None:  # xrs.go:236-301
        d, p = self.d, self.p
        if len(need) == 1 and need[0] < d:
            return self.reconst_one(vects, need[0])
        self._check_size(vects[0])
        if len(vects) != d + p:
            raise XRSError("illegal vects number")
        half = len(vects[0]) // 2
        a_vects = [v[:half] for v in vects]
        a_lost = [i for i in range(d + p) if i not in dp_has]
        self.rs_reconst(a_vects, dp_has, a_lost)
        self.retrieve_rs(vects, dp_has)
        b_vects = [v[half:] for v in vects]
        self.rs_reconst(b_vects, dp_has, need)
        pn = [i for i in need if i >= d]  # rs.SplitNeedReconst [dep]
        if len(pn) == 1 and pn[0] == d:
            return
        for i in pn:
            if i != d:
                for ai in self.xor_set.get(i, []):
                    vects[i][half:] ^= vects[ai][:half]

    def update(self, old, new, row: int, parity) -> None:  # xrs.go:324-346
        self._check_size(old)
        if row < 0 or row >= self.d:
            raise XRSError(f"illegal data index: {row}")
        delta = old ^ new
        for r in range(self.p):
            parity[r] ^= MUL[int(self.gen[self.d + r, row])][delta]
        _, b_need = self.get_need_vects(row)
        half = len(old) // 2
        parity[b_need[1] - self.d][half:] ^= delta[:half]

    def replace(self, data, rows, parity) -> None:  # xrs.go:363-387
        self._check_size(data[0])
        if len(rows) > self.d:
            raise XRSError("illegal vects number")
        for r in rows:
            if r < 0 or r >= self.d:
                raise XRSError(f"illegal data index: {r}")
        for r in range(self.p):
            for i, row in enumerate(rows):
                parity[r] ^= MUL[int(self.gen[self.d + r, row])][data[i]]
        half = len(data[0]) // 2
        for i, row in enumerate(rows):
            _, b_need = self.get_need_vects(row)
            parity[b_need[1] - self.d][half:] ^= data[i][:half]


def make_xor_set(d: int, p: int) -> dict:
    """xrs.go:77-100 (round robin of data i over parity d+1 .. d+p-1)."""
    m = {i: [] for i in range(d + 1, d + p)}
    j = d + 1
    for i in range(d):
        if j > d + p - 1:
            j = d + 1
        m[j].append(i)
        j += 1
    return {k: v for k, v in m.items() if v}


def make_xor_set_old(d: int, p: int) -> dict:
    """xrs_test.go:83-99 makeXORSetOld (the legacy algorithm the test compares to)."""
    m: dict = {}
    a = 0
    while a != d:
        for i in range(d + 1, d + p):
            if a == d:
                break
            m.setdefault(i, []).append(a)
            a += 1
    return m
