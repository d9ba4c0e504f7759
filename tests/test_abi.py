"""CPU tests of the C ABI (include/xrs_hip.h): the library loads, exports every
declared symbol, and its host logic (New, XORSet, GetNeedVects, generator,
error texts) matches the reference.  No kernel is launched here."""
import ctypes
import os
import re

import numpy as np
import pytest

import xrs_amd
from oracle.xrs_oracle import XRS as PyXRS
from oracle.xrs_oracle import make_xor_set_old

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "xrs_hip.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(xrs_[a-z0-9_]+)\s*\(", src)))


def gpu_present():
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        n = ctypes.c_int(0)
        return hip.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0
    except OSError:
        return False


def test_exports_every_declared_symbol():
    syms = declared_symbols()
    assert len(syms) >= 20
    lib = ctypes.CDLL(xrs_amd.LIB_PATH)
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_version_mentions_gfx950():
    assert b"gfx950" in xrs_amd.lib().xrs_version()


def test_library_built_from_this_tree():
    """xrs_version() carries the digest of the sources the .so was built from
    (xrs_amd/csrc/version.cpp); it must equal the tree's digest, i.e. the
    shipped library is not stale (rebuild: make -C xrs_amd/csrc)."""
    built, tree = xrs_amd.library_source_hash(), xrs_amd.source_hash()
    assert re.fullmatch(r"[0-9a-f]{16}", tree)
    assert built == tree, f"libxrs_hip.so was built from sources {built}, the tree is {tree}"


def test_new_errors():
    with pytest.raises(xrs_amd.XRSError, match="^illegal parity$"):
        xrs_amd.XRS(12, 1)
    for d, p in [(0, 4), (-1, 2), (255, 2), (12, 0)]:
        with pytest.raises(xrs_amd.XRSError):
            xrs_amd.XRS(d, p)
    xrs_amd.XRS(254, 2)
    xrs_amd.XRS(1, 255)


def test_xor_set_and_need_vects_all_configs():
    """xrs_test.go:51-80 (makeXORSet == makeXORSetOld) and :124-156
    (aNeed + k == XORSet[bNeed[1]], New succeeds) for every d+p <= 256,
    through the product library's host logic."""
    for d in range(1, 256):
        for p in range(2, 257 - d):
            x = xrs_amd.XRS(d, p)
            assert x.xor_set == make_xor_set_old(d, p), (d, p)
            if p in (2, 3, 4, 7, 256 - d) or d < 8:
                xs = x.xor_set
                for i in range(d):
                    a, b = x.get_need_vects(i)
                    assert b[0] == d
                    assert sorted(a + [i]) == xs[b[1]]


def test_generator_matches_oracle():
    for d, p in [(12, 4), (5, 5), (10, 4), (1, 2), (200, 56)]:
        g = np.frombuffer(xrs_amd.XRS(d, p).gen_matrix, np.uint8).reshape(d + p, d)
        assert np.array_equal(g, PyXRS(d, p).gen)


def test_need_vects_12p4():
    x = xrs_amd.XRS(12, 4)
    assert x.xor_set == {13: [0, 3, 6, 9], 14: [1, 4, 7, 10], 15: [2, 5, 8, 11]}
    for k in range(12):
        a, b = x.get_need_vects(k)
        assert b == [12, 13 + k % 3]
        assert a == [i for i in range(k % 3, 12, 3) if i != k]
    with pytest.raises(xrs_amd.XRSError, match="^illegal data index: -1$"):
        x.get_need_vects(-1)


def test_error_messages_are_go_text():
    x = xrs_amd.XRS(12, 4)
    with pytest.raises(xrs_amd.XRSError, match="^vect size not even: 5$"):
        x.encode([np.zeros(5, np.uint8) for _ in range(16)])
    with pytest.raises(xrs_amd.XRSError, match="^vect size not even: 7$"):
        x.reconst_one([np.zeros(7, np.uint8) for _ in range(16)], 0)
    with pytest.raises(xrs_amd.XRSError, match="^illegal data index: 12$"):
        x.reconst_one([np.zeros(8, np.uint8) for _ in range(16)], 12)
    with pytest.raises(xrs_amd.XRSError, match="^illegal data index: 13$"):
        x.update(np.zeros(8, np.uint8), np.zeros(8, np.uint8), 13,
                 [np.zeros(8, np.uint8) for _ in range(4)])
    with pytest.raises(xrs_amd.XRSError, match="^illegal data index: 12$"):
        x.replace([np.zeros(8, np.uint8)], [12], [np.zeros(8, np.uint8) for _ in range(4)])
    with pytest.raises(xrs_amd.XRSError, match="^illegal vects$"):
        x.encode([np.zeros(8, np.uint8) for _ in range(15)])


def test_mismatched_vect_lengths_rejected_before_the_call():
    """Every vect must be as long as vects[0] (the C ABI reads / writes that
    many bytes of each): ADVICE r1.  The even-size rule is checked first."""
    x = xrs_amd.XRS(12, 4)
    v = [np.zeros(64, np.uint8) for _ in range(16)]
    v[13] = np.zeros(32, np.uint8)
    for call in (lambda: x.encode(v), lambda: x.reconst_one(v, 0),
                 lambda: x.reconst(v, list(range(12)), [12, 13]),
                 lambda: x.update(np.zeros(64, np.uint8), np.zeros(62, np.uint8), 0,
                                  [np.zeros(64, np.uint8)] * 4),
                 lambda: x.update(np.zeros(64, np.uint8), np.zeros(64, np.uint8), 0,
                                  [np.zeros(64, np.uint8)] * 3 + [bytearray(65)]),
                 lambda: x.replace([np.zeros(64, np.uint8), np.zeros(128, np.uint8)], [0, 1],
                                   [np.zeros(64, np.uint8)] * 4)):
        with pytest.raises(xrs_amd.XRSError, match="^illegal vects$"):
            call()
    odd = [np.zeros(63, np.uint8) for _ in range(16)]
    odd[2] = np.zeros(10, np.uint8)
    with pytest.raises(xrs_amd.XRSError, match="^vect size not even: 63$"):
        x.encode(odd)


@pytest.mark.skipif(gpu_present(), reason="checks the no-GPU behaviour")
def test_compute_without_gpu_fails_loudly():
    x = xrs_amd.XRS(12, 4)
    with pytest.raises(xrs_amd.XRSError, match="no gpu device"):
        x.encode([np.zeros(8, np.uint8) for _ in range(16)])
    with pytest.raises(xrs_amd.XRSError, match="no gpu device"):
        x.encode_batched(1 << 20, 4096, 4096, 65536, 1)
    with pytest.raises(xrs_amd.XRSError, match="no gpu device"):
        xrs_amd.XRSGroup(12, 4, [0])


def test_single_hip_runtime():
    """The codec library shares torch's HIP runtime (xrs_amd/__init__.py
    _load): one libamdhip64 mapped, whichever of the two is imported first."""
    import subprocess
    import sys
    code = ("import xrs_amd, torch; rt = xrs_amd.hip_runtimes(); "
            "assert len(rt) == 1, rt; print(rt[0])")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stderr[-2000:]


def test_batch_layout_offset():
    """xrs_batch_layout: the strides of xrs_batch_strides and the base offset
    that puts shard 0's b-half (vect[S/2:]) on 16 B: 0 for sizes that are
    multiples of 32 (profiles/r03_layout_odd.log)."""
    for size in (2, 4, 34, 1026, 4096, 4098, 4100, 4126, 65538, 1 << 20, (1 << 20) + 2, 8 << 20):
        sh, st, off = xrs_amd.batch_layout(size, 16)
        assert (sh, st) == xrs_amd.batch_strides(size, 16)
        assert 0 <= off < 16 and (off + size // 2) % 16 == 0, size
    assert xrs_amd.batch_layout(4096, 16)[2] == 0 and xrs_amd.batch_layout(4100, 16)[2] == 14
    assert xrs_amd.batch_layout((1 << 20) + 2, 16)[2] == 15
    with pytest.raises(xrs_amd.XRSError):
        xrs_amd.batch_layout(4096, 0)
    # strides that would not fit in size_t are refused (no wrap-around)
    for size in (1 << 62, (1 << 64) - 2):
        with pytest.raises(xrs_amd.XRSError):
            xrs_amd.batch_strides(size, 16)
    sh, st = xrs_amd.batch_strides(1 << 58, 16)
    assert sh == (1 << 58) + 4352 and st >= 16 * sh


def test_batch_strides_recommendation():
    """xrs_batch_strides (codec.cpp): shards back to back below 4 MiB, odd
    sizes back to back below 32 KiB, 16-rounded from there, a 4 KiB + 256 B
    pad from 4 MiB up (profiles/r02_stride_probe.log, r01_order_ab.log); the
    stripe stride rounded up to a power of two when that costs at most 1/7
    of the packed stripe (profiles/r02_layout_*.log)."""
    cases = {4096: 4096, 4100: 4100, 2: 2, 1026: 1026, 65536: 65536, 65538: 65552,
             1 << 20: 1 << 20, (1 << 20) + 2: (1 << 20) + 16, 8 << 20: (8 << 20) + 4352}
    for size, shard in cases.items():
        assert xrs_amd.batch_strides(size, 16) == (shard, 16 * shard), size
    # 12+3: 15 x 4 KiB = 60 KiB -> 64 KiB (1/15 more); 10+4: 56 -> 64 KiB
    # (exactly 1/7); 16+4: 80 KiB stays (128 KiB would cost 3/5 more)
    assert xrs_amd.batch_strides(4096, 15) == (4096, 65536)
    assert xrs_amd.batch_strides(4096, 14) == (4096, 65536)
    assert xrs_amd.batch_strides(4096, 20) == (4096, 20 * 4096)
    assert xrs_amd.batch_strides(4096, 9) == (4096, 9 * 4096)
    assert xrs_amd.batch_strides(1 << 20, 15) == (1 << 20, 16 << 20)
    assert xrs_amd.batch_strides(4 << 20, 15) == ((4 << 20) + 4352, 64 << 20)
    assert xrs_amd.batch_strides(4100, 15) == (4100, 65536)  # odd sizes too (+3..6%)
    assert xrs_amd.batch_strides(4100, 16) == (4100, 16 * 4100)
    assert xrs_amd.batch_strides(4000, 16) == (4000, 65536)
    for size in (1, 2, 100, 4096, 5000, 1 << 20, 3 << 20, 9 << 20):
        for n in range(1, 40):
            sh, st = xrs_amd.batch_strides(size, n)
            assert sh >= size and n * sh <= st <= n * sh * 8 // 7, (size, n)
