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
import sys
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


def test_no_sgpr_spills_in_product(ks):
    """Round 6: the product library holds only kernels
    that keep every register in registers — the stencil tiles whose kernels
    spilled SGPRs (2- and 4-row dword rings, 4-row and private-ring 2-row x4
    tiles, prefetch depth 3 at 2 rows) are compiled in the tuning build only
    (-DLHPC_TUNING_ENV); the product refuses them with LHPC_ERR_UNSUPPORTED."""
    bad = {n: r["sgpr_spill_count"] for n, r in ks.items() if r["sgpr_spill_count"]}
    assert not bad, f"{len(bad)} kernels spill SGPRs: {sorted(bad)[:4]}"
    s7 = [n for n in ks if "k_stencil7" in n]
    assert 0 < len(s7) <= 64, len(s7)


def test_product_build_tag():
    """lhpc_build_flags() is 0 for the product library and has the debug bit
    for the debug build."""
    import ctypes
    prod = ctypes.CDLL(LIB)
    assert prod.lhpc_build_flags() == 0
    dbg = os.path.join(ROOT, "libhpc_amd", "_lib_debug", "liblhpc.so")
    if os.path.exists(dbg):
        assert ctypes.CDLL(dbg).lhpc_build_flags() & 2


def _gpurun_ignored(rel, patterns):
    rel = "./" + rel
    return any(rel == p or rel.startswith(p.rstrip("/") + "/") for p in patterns if p.startswith("./"))


def test_no_probe_build_travels():
    """Of the lhpc libraries in the tree, none that goes to the GPU box is a
    timing-only probe build (lhpc_build_flags & LHPC_BUILD_PROBE), and the
    only one with flags 0 is the product library.
    Tuning and probe build directories are listed in .gpurunignore."""
    import ctypes
    pats = [ln.strip() for ln in open(os.path.join(ROOT, ".gpurunignore")) if ln.strip() and not ln.startswith("#")]
    travel = {}
    for d, _, files in os.walk(os.path.join(ROOT, "libhpc_amd")):
        for f in files:
            if f.startswith("liblhpc") and f.endswith(".so") and "probe" not in f:
                rel = os.path.relpath(os.path.join(d, f), ROOT)
                if not _gpurun_ignored(rel, pats):
                    travel[rel] = ctypes.CDLL(os.path.join(ROOT, rel)).lhpc_build_flags()
    assert not {r: f for r, f in travel.items() if f & 4}, travel
    assert [r for r, f in travel.items() if f == 0] == ["libhpc_amd/_lib/liblhpc.so"], travel
    assert _gpurun_ignored("libhpc_amd/_lib_tuning/liblhpc.so", pats)


def test_loader_refuses_probe_build(tmp_path):
    """LHPC_LIB_PATH naming a timing-only probe build (lhpc_build_flags has
    LHPC_BUILD_PROBE) fails the import unless LHPC_ALLOW_PROBE_BUILD=1."""
    src = tmp_path / "probe.c"
    src.write_text("int lhpc_build_flags(void) { return 4; }\n")
    so = tmp_path / "liblhpc.so"
    subprocess.run(["gcc", "-shared", "-fPIC", str(src), "-o", str(so)], check=True)
    code = "import libhpc_amd"
    env = dict(os.environ, LHPC_LIB_PATH=str(so))
    env.pop("LHPC_ALLOW_PROBE_BUILD", None)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "timing-only probe build" in r.stderr, r.stderr[-2000:]
