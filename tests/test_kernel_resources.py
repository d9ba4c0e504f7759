"""Register and scratch budgets of the gfx950 kernels, read from the code
object inside xrs_amd/libxrs_hip.so (no GPU needed): the AMDGPU metadata
notes give each kernel's VGPR / AGPR count and private (scratch) segment.

A bandwidth kernel here holds every row it reads in registers, so its wave
occupancy is set by its VGPR count; a source change that pushes the headline
Encode from 170 VGPRs past 256 (AGPRs in use, one wave per SIMD) cost 26-43%
on the padded shapes before it was caught (profiles/r03_pad_ab.log).  These
budgets pin the headline instantiations and the staged Reconst kernels."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "xrs_amd", "libxrs_hip.so")
LLVM = "/opt/rocm/llvm/bin"

# (symbol regex, max VGPRs) -- the kernels bench.py and smoke() run.  A bound
# is the count up to which a compute unit still holds as many of the kernel's
# blocks as it does now (512 VGPRs per SIMD lane, allocated in 8s): 128 keeps
# four waves per SIMD, which is two 512-lane blocks (enc_ws) or one 1024-lane
# block (staged_wsp); 176 keeps the pair kernel's two waves per SIMD.
BUDGETS = [
    (r"pair_kernelILi4ELi12ELb0ELb1ELi128ELb1E", 176),   # Encode 12+4 @ 1 MiB (dominant, 170)
    (r"enc_ws_kernelILi12ELi256EE", 128),                # Encode 12+4 @ 4 KiB (102)
    (r"enc_ws_kernelILi10ELi256EE", 128),                # Encode 10+4 @ 4 KiB (94)
    (r"enc_ws_kernelILi8ELi256EE", 128),                 # Encode 8+4 @ 4 KiB (89)
    (r"rows_kernelILi2ELi12ELi4ELb0ELb1ELi1024E", 128),  # ReconstOne @ 1 MiB (1024-thread blocks, 94)
    (r"rows_kernelILi2ELi12ELi4ELb0ELb1ELi256E", 128),   # ReconstOne @ 4 KiB (96)
    (r"staged_wsp_kernelILi12ELi14ELi2ELi2ELi512EE", 128),  # 2 lost @ 1 MiB (106)
    (r"staged_ws_kernelILi12ELi14ELi2ELi2ELi256ELi1E", 128),
    (r"staged_ws_kernelILi12ELi15ELi1ELi1ELi256ELi1E", 128),
]


def _code_objects(tmp_path):
    for tool in ("objcopy",):
        if not shutil.which(tool):
            pytest.skip(f"{tool} not available")
    if not os.path.exists(os.path.join(LLVM, "llvm-readelf")):
        pytest.skip("ROCm LLVM tools not available")
    fat = tmp_path / "fat.bin"
    # (an output file is named so that objcopy leaves the library untouched:
    # with none it rewrites its input in place)
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", LIB,
                    str(tmp_path / "discard.so")], check=True)
    # The library links one offload bundle per kernels.hip build part
    # (XRS_PART): the section holds them back to back, each opening with the
    # bundle magic.
    data = fat.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts, i = [], data.find(magic)
    while i >= 0:
        starts.append(i)
        i = data.find(magic, i + 1)
    assert starts, "no offload bundle in .hip_fatbin"
    cos = []
    for n, (a, b) in enumerate(zip(starts, starts[1:] + [len(data)])):
        part = tmp_path / f"part{n}.bin"
        part.write_bytes(data[a:b])
        co = tmp_path / f"k{n}.co"
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}",
                        f"--output={co}", "--unbundle"], check=True)
        cos.append(co)
    return cos


def _notes(tmp_path):
    return "\n".join(subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", str(co)],
                                    capture_output=True, text=True, check=True).stdout
                     for co in _code_objects(tmp_path))


def _kernels(txt):
    starts = [m.start() for m in re.finditer(r"\.agpr_count:", txt)] + [len(txt)]
    out = {}
    for a, b in zip(starts, starts[1:]):
        blk = txt[a:b]

        def field(k):
            m = re.search(r"\.%s:\s+(\S+)" % k, blk)
            return m.group(1) if m else None
        sym = field("symbol")
        if sym:
            out[sym] = {"vgpr": int(field("vgpr_count")), "agpr": int(field("agpr_count")),
                        "scratch": int(field("private_segment_fixed_size"))}
    return out


def test_kernel_register_budgets(tmp_path):
    ks = _kernels(_notes(tmp_path))
    assert len(ks) > 100  # every instantiation is in the code object
    for pat, vmax in BUDGETS:
        hits = {s: v for s, v in ks.items() if re.search(pat, s)}
        assert hits, pat
        for s, v in hits.items():
            assert v["agpr"] == 0 and v["vgpr"] <= vmax, (s, v)
    # No kernel a default dispatch can launch spills to scratch.  The two
    # that do are A/B-only: the 5-wave-capped staged kernel (T = 128, OCC =
    # 5: XRS_STAGED_WS=128o5) and 1024-thread ReconstOne blocks for 20+4
    # (26-27 rows; the launcher takes 1024-thread blocks only up to 22 rows,
    # XRS_ROWS_BLOCK=1024 forces them).
    ab_only = re.compile(r"staged_ws_kernelILi12ELi1[234]ELi[34]ELi[34]ELi128ELi5E|"
                         r"rows_kernelILi2ELi20ELi[67]ELb0ELb1ELi1024E")
    spills = {s: v for s, v in ks.items() if v["scratch"] and not ab_only.search(s)}
    assert not spills, list(spills)[:5]


def test_persistent_slot_reset_order(tmp_path):
    """The persistent staged Reconst kernel hands its counter slot back with
    no fence (kernels.hip, staged_wsp_kernel): the last block swaps both
    counters to 0 and then clears the slot's pinned host busy word with a
    relaxed system-scope store.  The order is only right if both swaps have
    returned (been performed at L2) before that store issues; otherwise the
    host could give the slot to the next launch while its counters still
    hold this launch's values, and that launch would skip tiles (wrong
    Reconst output, xrs.go:236-320).  Pin it in the shipped code object:
    two returning global_atomic_swap, then s_waitcnt vmcnt(0), then the
    sc0 sc1 (system-scope) global_store_dword, with no other memory
    instruction in between."""
    objdump = os.path.join(LLVM, "llvm-objdump")
    if not os.path.exists(objdump):
        pytest.skip("llvm-objdump not available")
    pat = re.compile(r"_Z\S*staged_wsp_kernelILi12ELi14ELi2ELi2ELi512EE\S*")
    checked = 0
    for co in _code_objects(tmp_path):
        syms = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "-s", "--wide", str(co)],
                              capture_output=True, text=True, check=True).stdout
        names = sorted({m.group(0) for m in pat.finditer(syms)
                        if "." not in m.group(0)})
        for sym in names:
            dis = subprocess.run([objdump, "-d", f"--disassemble-symbols={sym}", str(co)],
                                 capture_output=True, text=True, check=True).stdout
            ins = [ln.split("//")[0].strip() for ln in dis.splitlines()]
            ins = [i for i in ins if i and not i.endswith(">:") and not i.startswith("Disassembly")]
            swaps = [n for n, i in enumerate(ins) if i.startswith("global_atomic_swap")]
            assert len(swaps) == 2, (sym, [ins[n] for n in swaps])
            for n in swaps:  # returning form: sc0 (glc) set
                assert re.search(r"\bsc0\b", ins[n]), ins[n]
            a, b = swaps
            assert all(not ins[n].startswith(("global_", "flat_", "buffer_"))
                       for n in range(a + 1, b)), ins[a:b + 1]
            tail = ins[b + 1:]
            st = next(n for n, i in enumerate(tail) if i.startswith("global_store_dword "))
            assert re.search(r"\bsc0 sc1\b", tail[st]), tail[st]  # the system-scope busy store
            between = tail[:st]
            assert any(re.match(r"s_waitcnt .*vmcnt\(0\)", i) for i in between), between
            assert not any(i.startswith(("global_", "flat_", "buffer_")) for i in between), between
            checked += 1
    assert checked >= 1
