"""CPU: the built libsfmfeat.so contains no instruction form known to return wrong results
on gfx950 while an MFMA of another wave runs on the same SIMD.

tools/pk_mfma_hazard.hip measured it (profiles/r04_pk_mfma_hazard.txt, DESIGN.md §7
*Co-residency*): a packed-FP32 instruction (`v_pk_fma_f32`, `v_pk_mul_f32`, `v_pk_add_f32`)
whose low result reads src1's high half (op_sel bit 1 set) returns wrong low results in lanes
48-63 beside a registers-only MFMA co-runner; the forms without it (no op_sel, src0's or
src2's high half, src1's low half broadcast by op_sel_hi) measured clean.  The product runs Harris (packed fmas) and the matcher
(MFMA) of two batches at once, so a compiler or source change that brings the form back must
fail here, on the CPU, before any GPU run.

The device code objects are read from the library's .hip_fatbin section (one offload bundle
per translation unit) with the ROCm LLVM tools; the test skips when they are missing."""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "sfmfromscratch_amd", "lib", "libsfmfeat.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# (instruction, op_sel pattern) pairs measured to misbehave beside MFMA: every packed-FP32
# form whose low result takes src1's high half (profiles/r04_pk_mfma_hazard.txt)
FORBIDDEN = [("v_pk_fma_f32", re.compile(r"op_sel:\[[01],1,[01]\]")),
             ("v_pk_mul_f32", re.compile(r"op_sel:\[[01],1\]")),
             ("v_pk_add_f32", re.compile(r"op_sel:\[[01],1\]"))]


def _device_elfs(tmp_path) -> list:
    """The library's device code objects (one per translation unit), unbundled into tmp_path."""
    objcopy = shutil.which("objcopy")
    bundler, objdump = os.path.join(LLVM, "clang-offload-bundler"), os.path.join(LLVM, "llvm-objdump")
    if not (os.path.exists(LIB) and objcopy and os.path.exists(bundler) and os.path.exists(objdump)):
        pytest.skip("library or ROCm LLVM tools not available")
    fb = tmp_path / "fatbin.bin"
    subprocess.run([objcopy, "-O", "binary", "--only-section=.hip_fatbin", LIB, str(fb)], check=True)
    data = fb.read_bytes()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    assert starts, "no offload bundle in .hip_fatbin"
    out = []
    for n, i in enumerate(starts):
        j = starts[n + 1] if n + 1 < len(starts) else len(data)
        b, e = tmp_path / f"b{n}.bin", tmp_path / f"b{n}.elf"
        b.write_bytes(data[i:j])
        subprocess.run([bundler, "--unbundle", "--type=o", f"--input={b}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={e}"], check=True)
        out.append(str(e))
    return out


def _device_asm(tmp_path) -> str:
    objdump = os.path.join(LLVM, "llvm-objdump")
    return "\n".join(subprocess.run([objdump, "-d", "--mcpu=gfx950", e], check=True, capture_output=True,
                                    text=True).stdout for e in _device_elfs(tmp_path))


def _kernel_meta(tmp_path) -> dict:
    """Per kernel symbol: static LDS bytes, VGPRs and scratch bytes per lane, from the code
    objects' AMDGPU metadata notes.  The keys of a kernel's map print in sorted order, starting
    with .agpr_count; .vgpr_count follows .name, so a record closes at the next map's start."""
    readelf = os.path.join(LLVM, "llvm-readelf")
    keys = {"group_segment_fixed_size": "lds", "vgpr_count": "vgpr", "private_segment_fixed_size": "scratch",
            "name": "name"}
    meta = {}
    for e in _device_elfs(tmp_path):
        notes = subprocess.run([readelf, "--notes", e], check=True, capture_output=True, text=True).stdout
        cur = {}
        for line in notes.splitlines() + ["  - .agpr_count: 0"]:
            if re.match(r"^\s*-\s*\.agpr_count:", line):
                if "name" in cur:
                    meta[cur.pop("name")] = cur
                cur = {}
            for k, v in keys.items():
                m = re.search(r"^\s*-?\s*\.%s:\s*(\S+)" % k, line)
                if m and v not in cur:
                    cur[v] = m.group(1) if v == "name" else int(m.group(1))
    return meta


def _kernel_lds(tmp_path) -> dict:
    """Static LDS bytes per kernel symbol."""
    return {k: v["lds"] for k, v in _kernel_meta(tmp_path).items()}


def test_half_cu_sweep_fits_beside_one_harris_workgroup(tmp_path):
    """The half-CU matcher sweep (k_match_mfma<3>) exists to share a CU with one k_harris
    workgroup of the other batch: their LDS together must fit the CU's 160 KB.
    Read from the built code objects, so a Harris form that grows its LDS (e.g. another
    histogram copy) cannot silently lose the co-residency."""
    lds = _kernel_lds(tmp_path)
    harris = [v for k, v in lds.items() if k.startswith("_ZN3sfm8k_harrisILi7ELb1ELi0ELi0E")]
    sweep3 = [v for k, v in lds.items() if k.startswith("_ZN3sfm12k_match_mfmaILi3ELi0E")]
    assert len(harris) == 1 and len(sweep3) == 1, (harris, sweep3)
    assert harris[0] + sweep3[0] <= 160 * 1024, f"k_harris {harris[0]} B + half-CU sweep {sweep3[0]} B > 160 KB"


def test_select_workgroup_fits_beside_one_harris_workgroup(tmp_path):
    """k_select (one 1,024-thread workgroup per plane, mostly waiting on loads) runs on the aux
    stream while the other batch's k_harris holds the CUs.  Its LDS is sized per launch from k
    (select.hip select_lds_bytes) and its VGPRs are budgeted so that one select workgroup and one
    k_harris workgroup share a CU: LDS within 160 KB, and 4 select waves + 1 Harris wave per
    SIMD within the 512-entry register file (allocation granule 8), with no scratch spills."""
    meta = _kernel_meta(tmp_path)
    harris = [v for k, v in meta.items() if k.startswith("_ZN3sfm8k_harrisILi7ELb1ELi0ELi0E")]
    sel = [v for k, v in meta.items() if k.startswith("_ZN3sfm8k_selectE")]
    assert len(harris) == 1 and len(sel) == 1, (harris, sel)
    h, s = harris[0], sel[0]

    def alloc(v):
        return (v + 7) // 8 * 8

    assert s["scratch"] == 0, f"k_select spills {s['scratch']} B per lane"
    assert 4 * alloc(s["vgpr"]) + alloc(h["vgpr"]) <= 512, f"k_select {s['vgpr']} VGPRs x 4 + k_harris {h['vgpr']} > 512"
    k = 2500  # BASELINE's k: sel area next_pow2(k) keys, ties 2048, 4096-bin histogram, 1024 scan words
    sel_cap = max(2048, 1 << (k - 1).bit_length())
    dyn = sel_cap * 8 + 2048 * 8 + 4096 * 4 + 1024 * 4
    assert s["lds"] + dyn + h["lds"] <= 160 * 1024, f"k_select {s['lds'] + dyn} B + k_harris {h['lds']} B > 160 KB"


def test_no_packed_fma_with_src1_high_half_select(tmp_path):
    asm = _device_asm(tmp_path)
    assert "v_pk_fma_f32" in asm and "v_mfma" in asm  # the scan sees both kernels' code
    bad, kernel = [], None
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
        if m:
            kernel = m.group(1)
            continue
        for op, pat in FORBIDDEN:
            if op in line and pat.search(line):
                bad.append(f"{kernel}: {line.split('//')[0].strip()}")
    assert not bad, f"{len(bad)} hazardous instructions, e.g. {bad[:3]}"


def test_harris_window_at_its_fma_floor_and_non_window_valu_bounded():
    """The shipped product Harris kernel (k_harris<7, true, 0, 0>) from the built library's ISA
    (tools/isa_phases.py, static counts over the tile loop, interior and border branches both
    counted): the window is exactly the 49-tap fmaf contract's 16 px x 147 = 2352 fmas per
    tile-thread, and the instructions around it stay at most 1,000 per tile-wave (977 at the end
    of round 6; 607 on the interior path alone, profiles/r06_harris_isa_phases_interior.txt), so
    a compiler or source change that brings back round 5's overhead (the LDS tap reads, the
    scalar R epilogue: 918 on the interior path) fails here."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_phases as ip
    if not os.path.exists(LIB) or not os.path.exists(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("library or ROCm LLVM tools not available")
    _, ins = ip.kernel_body(ip.disassemble(LIB), "k_harrisILi7ELb1ELi0ELi0E")
    cnt, _, _, _, _, win, sc = ip.phase_counts(ins)
    assert 2 * win + sc == 16 * 147, (win, sc)
    non_window = sum(cnt.values()) - cnt["window fmas"]
    assert non_window <= 1000, f"{non_window} non-window VALU per tile-wave"
