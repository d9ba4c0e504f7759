"""Generate tests/golden/xrs_golden.npz (committed) -- run from the repo root:

    python tests/golden/make_golden.py

Vectors come from the C restatement (oracle/xrs_oracle.c) and every one is
re-derived with the independent numpy restatement (oracle/xrs_oracle.py);
the script refuses to write the file if the two disagree or if either fails
the reference's known-answer test (xrs_test.go:102-122).  Inputs are seeded
(numpy PCG64, seed 0x5EED), unlike the reference's time-seeded tests.

Cases (12+4 unless noted), S in {2, 64, 1026, 4096}:
  kat            5+5 KAT of xrs_test.go:108-115 (in/out)
  enc_S          Encode: data in, full stripe out
  rc{i}_S        general Reconst (xrs.go:236): dp_has, need, buffers in/out
                 (out includes the reference's side effects: a-halves of all
                 lost vects, surviving parity b-halves left in RS form)
  up_S_row{r}    Update (xrs.go:324): old/new/parity in, parity out
  rp_S_n{n}_{z}  Replace (xrs.go:363) with n rows, z = tozero|fromzero
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle.oracle_c import OracleXRS  # noqa: E402
from oracle.xrs_oracle import XRS as PyXRS  # noqa: E402

SIZES = (2, 64, 1026, 4096)
D, P = 12, 4
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "xrs_golden.npz")


def both(fn_c, fn_py, bufs_c, bufs_py):
    fn_c(bufs_c)
    fn_py(bufs_py)
    for a, b in zip(bufs_c, bufs_py):
        if not np.array_equal(a, b):
            raise SystemExit("C and numpy restatements disagree -- not writing goldens")


def main():
    rng = np.random.Generator(np.random.PCG64(0x5EED))
    out = {}
    # KAT
    kat_in = np.array([[0, 0], [4, 7], [2, 4], [6, 9], [8, 11]] + [[0, 0]] * 5, dtype=np.uint8)
    kat_exp = np.array([[0, 0], [4, 7], [2, 4], [6, 9], [8, 11], [97, 156], [173, 117],
                        [218, 110], [107, 59], [110, 153]], dtype=np.uint8)
    for cls in (OracleXRS, PyXRS):
        v = [r.copy() for r in kat_in]
        cls(5, 5).encode(v)
        if not np.array_equal(np.stack(v), kat_exp):
            raise SystemExit(f"{cls.__name__} fails the reference KAT")
    out["kat_in"], out["kat_out"] = kat_in, kat_exp

    xc, xp = OracleXRS(D, P), PyXRS(D, P)
    for S in SIZES:
        data = rng.integers(0, 256, size=(D + P, S), dtype=np.uint8)
        data[D:] = 0
        vc = [r.copy() for r in data]
        vp = [r.copy() for r in data]
        both(xc.encode, xp.encode, vc, vp)
        enc = np.stack(vc)
        out[f"enc_S{S}_in"] = data[:D].copy()
        out[f"enc_S{S}_out"] = enc

        # general Reconst: lost sets of size 0..4, need = prefixes
        cases = [([], []), ([0, 1], [0, 1]), ([13, 2], [13]), ([12, 14, 5], [14, 5, 12]),
                 ([3, 15, 9, 13], [15, 3]), ([15, 14], []), ([7, 11, 12, 13], [7, 11, 12, 13]),
                 ([4], [4, 14]), ([0, 13, 14, 15], [13, 14, 15])]
        for i, (lost, need) in enumerate(cases):
            has = [j for j in range(D + P) if j not in lost]
            inb = enc.copy()
            for j in lost:  # lost vects hold garbage
                inb[j] = rng.integers(0, 256, size=S, dtype=np.uint8)
            vc = [r.copy() for r in inb]
            vp = [r.copy() for r in inb]
            both(lambda v: xc.reconst(v, has, need), lambda v: xp.reconst(v, has, need), vc, vp)
            for t in need:
                if not np.array_equal(vc[t], enc[t]):
                    raise SystemExit(f"reconst case {i} did not rebuild vect {t}")
            out[f"rc{i}_S{S}_has"] = np.array(has, dtype=np.int32)
            out[f"rc{i}_S{S}_need"] = np.array(need, dtype=np.int32)
            out[f"rc{i}_S{S}_in"] = inb
            out[f"rc{i}_S{S}_out"] = np.stack(vc)

        # Update, every row
        for row in range(D):
            new = rng.integers(0, 256, size=S, dtype=np.uint8)
            pc = [r.copy() for r in enc[D:]]
            pp = [r.copy() for r in enc[D:]]
            xc.update(enc[row], new, row, pc)
            xp.update(enc[row], new, row, pp)
            if not all(np.array_equal(a, b) for a, b in zip(pc, pp)):
                raise SystemExit("update mismatch")
            ref = enc.copy()
            ref[row] = new
            rv = [r.copy() for r in ref]
            xp.encode(rv)
            if not all(np.array_equal(a, b) for a, b in zip(pc, rv[D:])):
                raise SystemExit("update != re-encode")
            out[f"up_S{S}_row{row}_new"] = new
            out[f"up_S{S}_row{row}_out"] = np.stack(pc)

        # Replace
        for n in (1, 4, 12):
            rows = [int(r) for r in rng.permutation(D)[:n]]
            for tozero in (True, False):
                full = enc.copy()
                base = full.copy()
                for r in rows:
                    base[r] = 0
                bv = [r.copy() for r in base]
                xp.encode(bv)
                par_in = (np.stack([r for r in full[D:]]) if tozero else np.stack(bv[D:]))
                par_exp = (np.stack(bv[D:]) if tozero else full[D:].copy())
                datarows = np.stack([full[r] for r in rows])
                pc = [r.copy() for r in par_in]
                pp = [r.copy() for r in par_in]
                xc.replace(list(datarows), rows, pc)
                xp.replace(list(datarows), rows, pp)
                if not all(np.array_equal(a, b) for a, b in zip(pc, pp)):
                    raise SystemExit("replace mismatch")
                if not np.array_equal(np.stack(pc), par_exp):
                    raise SystemExit("replace != re-encode")
                z = "tozero" if tozero else "fromzero"
                out[f"rp_S{S}_n{n}_{z}_rows"] = np.array(rows, dtype=np.int32)
                out[f"rp_S{S}_n{n}_{z}_in"] = par_in
                out[f"rp_S{S}_n{n}_{z}_out"] = np.stack(pc)
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: {len(out)} arrays, {os.path.getsize(OUT)} bytes")


if __name__ == "__main__":
    main()
