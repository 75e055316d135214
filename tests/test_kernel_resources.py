"""Register budget of every gfx950 kernel in the product library, read from
the code objects inside liblhpc.so (no GPU needed): no kernel spills to
scratch, and the hot kernels keep the occupancy their design assumes
(DESIGN.md §4).  The kernels' metadata come from the AMDHSA notes of each
translation unit's offload bundle (llvm-readelf --notes).  The library is
built with compressed bundles (hipcc --offload-compress: "CCOB" header, zstd),
which clang-offload-bundler unpacks; plain bundles are read directly."""
import os
import re
import struct
import subprocess
import tempfile

import pytest

from tests._support import ROOT

LIB = os.path.join(ROOT, "libhpc_amd", "_lib", "liblhpc.so")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
BUNDLER = "/opt/rocm/lib/llvm/bin/clang-offload-bundler"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
CMAGIC = b"CCOB"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _compressed_objects(data, td):
    """gfx950 code objects of the compressed bundles: header magic, u16
    version, u16 method, then (version ≥ 3) u64 total size, u64 uncompressed
    size, u64 hash; version 2 has u32 sizes"""
    objs, i = [], data.find(CMAGIC)
    while i >= 0:
        ver = struct.unpack_from("<H", data, i + 4)[0]
        tot = struct.unpack_from("<Q" if ver >= 3 else "<I", data, i + 8)[0]
        src, dst = os.path.join(td, f"b{i}.bin"), os.path.join(td, f"b{i}.co")
        open(src, "wb").write(data[i:i + tot])
        if TARGET in subprocess.run([BUNDLER, "--list", "--type=o", f"--input={src}"], capture_output=True,
                                    text=True, check=True).stdout:
            subprocess.run([BUNDLER, "--unbundle", "--type=o", f"--targets={TARGET}", f"--input={src}",
                            f"--output={dst}"], check=True)
            objs.append(open(dst, "rb").read())
        i = data.find(CMAGIC, i + tot)
    return objs


def _gfx950_objects(path, td):
    data = open(path, "rb").read()
    if data.find(CMAGIC) >= 0 and data.find(MAGIC) < 0:
        return _compressed_objects(data, td)
    objs, i = [], data.find(MAGIC)
    while i >= 0:
        n = struct.unpack_from("<Q", data, i + len(MAGIC))[0]
        off = i + len(MAGIC) + 8
        for _ in range(n):
            o, sz, tl = struct.unpack_from("<QQQ", data, off)
            off += 24
            triple = data[off:off + tl].decode()
            off += tl
            if "gfx950" in triple and sz:
                objs.append(data[i + o:i + o + sz])
        i = data.find(MAGIC, i + 1)
    return objs


def kernels(path=LIB):
    """name → {vgpr_count, vgpr_spill_count, sgpr_spill_count, private_segment_fixed_size}"""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for k, blob in enumerate(_gfx950_objects(path, td)):
            f = os.path.join(td, f"co{k}.elf")
            open(f, "wb").write(blob)
            notes = subprocess.run([READELF, "--notes", f], capture_output=True, text=True, check=True).stdout
            for ent in notes.split("\n  - ")[1:]:
                m = re.search(r"\.name:\s+(\S+)", ent)
                if not m:
                    continue
                rec = {}
                for key in ("vgpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size"):
                    v = re.search(r"\." + key + r":\s+(\d+)", ent)
                    rec[key] = int(v.group(1)) if v else None
                out[m.group(1)] = rec
    return out


@pytest.fixture(scope="module")
def ks():
    if not os.path.exists(READELF) or not os.path.exists(BUNDLER) or not os.path.exists(LIB):
        pytest.skip("llvm-readelf / clang-offload-bundler or the built library not available")
    k = kernels()
    assert len(k) > 40, "expected the product kernels in the code objects"
    return k


def test_no_kernel_spills_to_memory(ks):
    """No VGPR spills and no private (scratch) segment in any kernel.  SGPR
    spills are allowed: they land in VGPR lanes (v_writelane), not memory —
    only the large opt-in stencil tiles have them."""
    bad = {n: r for n, r in ks.items() if r["vgpr_spill_count"] or r["private_segment_fixed_size"]}
    assert not bad, f"kernels using scratch: {sorted(bad)[:5]}"


def test_hot_kernel_register_budgets(ks):
    """The XTILE iperm reduce runs 8 waves per SIMD (≤ 64 VGPRs) in fp32 —
    the round-1 A/B that made it the default (DESIGN.md §4 iperm reduce);
    the SELL kernel too (≤ 64, fp32 and fp64);
    the default stencil7 kernel (x4 ring, 2 rows × 4 blocks, LDS-shared
    halo) stays ≤ 128 VGPRs (4 waves per SIMD), under the dword ring's 150."""
    def pick(pat):
        return {n: r for n, r in ks.items() if re.search(pat, n)}
    red = pick(r"k_xtile_reduceIfLi[124]ELi512ELb1E")
    assert red and all(r["vgpr_count"] <= 64 for r in red.values()), red
    sell = pick(r"k_spmv_sellI[fd]E")  # SELL: 8 waves per SIMD, every gather of a row in flight
    assert len(sell) == 2 and all(r["vgpr_count"] <= 64 for r in sell.values()), sell
    s7 = pick(r"k_stencil7_buf4ILi2ELi4ELi[56]ELi2ELb[01]ELb1E")
    assert s7 and all(r["vgpr_count"] <= 128 for r in s7.values()), {n: r["vgpr_count"] for n, r in s7.items()}
