"""Generate tests/golden/xrs_golden_codecs.npz (committed) -- run from the repo root:

    python tests/golden/make_golden_codecs.py

Goldens for codecs other than 12+4 (the runtime-count kernels, output groups
and source chunks), made like make_golden.py: by the C restatement, each
re-derived by the independent numpy restatement; the script refuses to write
the file if they disagree.  Seeded (PCG64, 0xC0DEC).

Per codec d+p and S in {34, 2048}:
  d{d}p{p}_S{S}_enc_in / _enc_out          Encode
  d{d}p{p}_S{S}_rc{i}_has/_need/_in/_out   general Reconst (side effects in out)
  d{d}p{p}_S{S}_up_row/_up_old/_up_new/_up_in/_up_out   Update
  d{d}p{p}_S{S}_rp_rows/_rp_data/_rp_in/_rp_out         Replace
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle.oracle_c import OracleXRS  # noqa: E402
from oracle.xrs_oracle import XRS as PyXRS  # noqa: E402

CODECS = [(10, 4), (6, 3), (5, 5), (4, 2), (20, 4), (1, 2), (30, 6)]
SIZES = (34, 2048)
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "xrs_golden_codecs.npz")


def same(a, b, what):
    if not all(np.array_equal(x, y) for x, y in zip(a, b)):
        raise SystemExit(f"C and numpy restatements disagree on {what} -- not writing goldens")


def main():
    rng = np.random.Generator(np.random.PCG64(0xC0DEC))
    out = {}
    for d, p in CODECS:
        xc, xp = OracleXRS(d, p), PyXRS(d, p)
        n = d + p
        for S in SIZES:
            k = f"d{d}p{p}_S{S}_"
            data = rng.integers(0, 256, size=(n, S), dtype=np.uint8)
            data[d:] = 0
            vc, vp = [r.copy() for r in data], [r.copy() for r in data]
            xc.encode(vc)
            xp.encode(vp)
            same(vc, vp, k + "enc")
            enc = np.stack(vc)
            out[k + "enc_in"], out[k + "enc_out"] = data[:d].copy(), enc
            for i in range(2):
                lost = [int(t) for t in rng.permutation(n)[: int(rng.integers(1, p + 1))]]
                need = lost[: max(1, len(lost) - i)]
                has = [j for j in range(n) if j not in lost]
                inb = enc.copy()
                for j in lost:
                    inb[j] = rng.integers(0, 256, size=S, dtype=np.uint8)
                vc, vp = [r.copy() for r in inb], [r.copy() for r in inb]
                xc.reconst(vc, has, need)
                xp.reconst(vp, has, need)
                same(vc, vp, k + f"rc{i}")
                out[k + f"rc{i}_has"] = np.array(has, np.int32)
                out[k + f"rc{i}_need"] = np.array(need, np.int32)
                out[k + f"rc{i}_in"], out[k + f"rc{i}_out"] = inb, np.stack(vc)
            row = int(rng.integers(0, d))
            new = rng.integers(0, 256, size=S, dtype=np.uint8)
            pc, pp = [r.copy() for r in enc[d:]], [r.copy() for r in enc[d:]]
            xc.update(enc[row], new, row, pc)
            xp.update(enc[row], new, row, pp)
            same(pc, pp, k + "up")
            out[k + "up_row"] = np.array([row], np.int32)
            out[k + "up_old"], out[k + "up_new"] = enc[row].copy(), new
            out[k + "up_in"], out[k + "up_out"] = enc[d:].copy(), np.stack(pc)
            rows = [int(t) for t in rng.permutation(d)[: int(rng.integers(1, d + 1))]]
            rdata = rng.integers(0, 256, size=(len(rows), S), dtype=np.uint8)
            pc, pp = [r.copy() for r in enc[d:]], [r.copy() for r in enc[d:]]
            xc.replace(list(rdata), rows, pc)
            xp.replace([r.copy() for r in rdata], rows, pp)
            same(pc, pp, k + "rp")
            out[k + "rp_rows"] = np.array(rows, np.int32)
            out[k + "rp_data"] = rdata
            out[k + "rp_in"], out[k + "rp_out"] = enc[d:].copy(), np.stack(pc)
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: {len(out)} arrays")


if __name__ == "__main__":
    main()
