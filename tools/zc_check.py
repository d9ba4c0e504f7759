import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, xrs_amd
from oracle.oracle_c import OracleXRS
x, o = xrs_amd.XRS(12, 4), OracleXRS(12, 4)
rng = np.random.default_rng(1)
for size in (4096, 1030, 2):
    v = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(16)]
    a = [r.copy() for r in v]; b = [r.copy() for r in v]
    x.encode(a); o.encode(b)
    assert all(np.array_equal(p, q) for p, q in zip(a, b)), size
print("zero-copy encode ok")
