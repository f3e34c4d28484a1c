#!/usr/bin/env python3
"""Per-phase VALU instruction counts of one k_harris<7,true,0,0> tile iteration, from the
gfx950 disassembly of the built library (no GPU needed).

The tile loop runs from its first s_barrier to the backward branch that closes it.  Phases:
  sobel     the interior strip loop (edge tiles run the masked variant instead), weighted
            by its trip count ceil(PH * NS / NT)
  window    v_pk_fma_f32 / v_fmac_f32 / v_fma_f32 of the window sums (incl. the edge-row
            scalar fmas the compiler sank into the epilogue)
  products  v_pk_mul_f32 (Ix^2, Iy^2, IxIy per gradient row)
  R         v_mul/v_sub/v_add f32 of det - alpha tr^2
  hist      the digit-1 key and its LDS add (v_not/v_lshrrev/v_and, ds_add)
  masks     v_cmp / v_cndmask (the image tile's zero border, the histogram's bounds)
  other     addressing and moves (incl. the fused down2x3 block of wave 0, counted as if
            every wave ran it: an upper bound)
The phases are classified by opcode (the compiler interleaves R and the histogram with the
window's last rows), so the table is per tile-wave, not a timeline.
With --interior the tool compiles harris.hip itself with -DSFM_HARRIS_COUNT_INTERIOR (every
tile takes the interior-tile path: unmasked prefetch, tile copy, Sobel and epilogue), so the
static count of the tile loop is exactly the VALU count per tile-wave of an interior tile — the
tiles that do not touch the image border (all but 92 of the 510 per 1080p plane).  Without it
the loop holds both variants of each masked phase and the count is an upper bound.
usage: tools/isa_phases.py [--interior] [lib.so] [kernel-substring]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def disassemble(lib):
    with tempfile.TemporaryDirectory() as tmp:
        fb = os.path.join(tmp, "fb.bin")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fb], check=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        out = []
        for n, i in enumerate(starts):
            j = starts[n + 1] if n + 1 < len(starts) else len(data)
            b, e = os.path.join(tmp, f"b{n}.bin"), os.path.join(tmp, f"b{n}.elf")
            open(b, "wb").write(data[i:j])
            subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={b}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={e}"], check=True)
            out.append(subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", e],
                                      check=True, capture_output=True, text=True).stdout)
    return "\n".join(out)


def kernel_body(txt, pat):
    for f in re.split(r"\n(?=[0-9a-f]{16} <)", txt):
        m = re.match(r"[0-9a-f]{16} <(\S+)>:", f)
        if m and pat in m.group(1):
            ins = []
            for line in f.splitlines()[1:]:
                mm = re.match(r"\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-F]+):", line)
                if mm:
                    ins.append((mm.group(1), mm.group(2), int(mm.group(3), 16)))
            return m.group(1), ins
    raise SystemExit(f"no kernel matching {pat!r}")


def branch_target(ins, k):
    """Index of the target of the branch at k (simm16 words after the next instruction)."""
    op, args, addr = ins[k]
    off = int(args.split()[0])
    if off >= 32768:
        off -= 65536
    nxt = ins[k + 1][2] if k + 1 < len(ins) else addr + 4
    tgt = nxt + 4 * off
    for i, (_, _, a) in enumerate(ins):
        if a == tgt:
            return i
    return None


def interior_object(tmp, no_down=False):
    """harris.hip compiled with every tile on the interior path (the product flags + the macro);
    no_down: also without the fused pyramid block (run by the first wave only)."""
    src = os.path.join(ROOT, "sfmfromscratch_amd", "csrc", "harris.hip")
    out = os.path.join(tmp, "harris_interior%s.o" % ("_nd" if no_down else ""))
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                    "-fno-fast-math", "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize",
                    "-DSFM_HARRIS_COUNT_INTERIOR"] + (["-DSFM_HARRIS_COUNT_NO_DOWN"] if no_down else []) +
                   ["-c", src, "-o", out], check=True, stderr=subprocess.DEVNULL)
    return out


def phase_counts(ins):
    """(counter by phase, tile-loop bounds, barriers, Sobel loops, window pk / scalar fmas) of
    one kernel body."""
    # the tile loop: the backward branch with the largest span
    loop = None
    for k, (op, args, _) in enumerate(ins):
        if op in ("s_branch", "s_cbranch_execz", "s_cbranch_execnz", "s_cbranch_scc0", "s_cbranch_scc1",
                  "s_cbranch_vccz", "s_cbranch_vccnz"):
            t = branch_target(ins, k)
            if t is not None and t < k and (loop is None or k - t > loop[1] - loop[0]):
                loop = (t, k)
    a, b = loop
    bars = [k for k in range(a, b + 1) if ins[k][0] == "s_barrier"]
    # small backward loops inside the tile loop: the Sobel strip loops
    inner = []
    for k in range(a, b + 1):
        op = ins[k][0]
        if op.startswith("s_cbranch") or op == "s_branch":
            t = branch_target(ins, k)
            if t is not None and a < t < k and (k - t) < 400 and any(ins[i][0] == "v_pk_fma_f32" for i in range(t, k)):
                inner.append((t, k))
    NT, PH, NS = 256, 70, 18
    trips = -(-PH * NS // NT)
    cnt = collections.Counter()
    hist_ops = {"v_not_b32_e32", "v_lshrrev_b32_e32", "v_and_b32_e32", "v_xor3_b32", "v_ashrrev_i32_e32"}
    for k in range(a, b + 1):
        op = ins[k][0]
        if not op.startswith("v_") and not op.startswith("ds_add"):
            continue
        in_inner = [(t, e) for t, e in inner if t <= k <= e]
        if in_inner:
            # the interior variant (the shorter loop) is the one interior tiles run
            if in_inner[0] == min(inner, key=lambda te: te[1] - te[0]):
                cnt["sobel (x%d strips)" % trips] += trips
            continue
        if op in ("v_pk_fma_f32", "v_fmac_f32_e32", "v_fma_f32"):
            cnt["window fmas"] += 1
        elif op == "v_pk_mul_f32":
            cnt["products"] += 1
        elif op == "v_pk_add_f32":
            cnt["R (det - alpha tr^2)"] += 1
        elif op in ("v_mul_f32_e32", "v_sub_f32_e32", "v_add_f32_e32"):
            cnt["scalar f32 (R / fused pyramid)"] += 1
        elif op in hist_ops or op.startswith("ds_add"):
            cnt["histogram key + LDS add"] += 1
        elif op.startswith(("v_cmp", "v_cndmask")):
            cnt["masks (tile copy, hist bounds)"] += 1
        else:
            cnt["addressing / moves"] += 1
    win = sum(1 for k in range(a, b + 1) if ins[k][0] == "v_pk_fma_f32" and not any(t <= k <= e for t, e in inner))
    sc = sum(1 for k in range(a, b + 1) if ins[k][0] in ("v_fmac_f32_e32", "v_fma_f32"))
    return cnt, (a, b), bars, inner, trips, win, sc


def main():
    args = [a for a in sys.argv[1:] if a != "--interior"]
    interior = "--interior" in sys.argv[1:]
    pat = args[1] if len(args) > 1 else "k_harrisILi7ELb1ELi0ELi0E"
    if interior:
        tmpd = tempfile.TemporaryDirectory()
        name, ins = kernel_body(disassemble(interior_object(tmpd.name)), pat)
        _, ins_nd = kernel_body(disassemble(interior_object(tmpd.name, no_down=True)), pat)
    else:
        lib = args[0] if args else os.path.join(ROOT, "sfmfromscratch_amd", "lib", "libsfmfeat.so")
        name, ins = kernel_body(disassemble(lib), pat)
    cnt, (a, b), bars, inner, trips, win, sc = phase_counts(ins)
    if interior:
        # the fused pyramid block runs in the first wave of the four only: its instructions (the
        # difference to the build without it) count 1/4 per tile-wave
        cnt_nd = phase_counts(ins_nd)[0]
        down = collections.Counter({k: cnt[k] - cnt_nd.get(k, 0) for k in cnt})
        cnt = collections.Counter({k: cnt_nd.get(k, 0) + down[k] / 4.0 for k in cnt})
        print(f"(interior tiles; the fused-pyramid block, {sum(down.values())} VALU in wave 0 only, counted 1/4)")
    tot = sum(cnt.values())
    print(f"{name}: tile loop {b - a + 1} instructions, {len(bars)} barriers, sobel loops {len(inner)} "
          f"(trip count {trips})")
    print(f"{'phase':30s} {'VALU/tile-wave':>14s} {'share':>7s}")
    for k, v in sorted(cnt.items(), key=lambda kv: -kv[1]):
        print(f"{k:30s} {v:14.1f} {v / tot:7.1%}")
    print(f"{'total':30s} {tot:14.1f}")
    print(f"{'non-window':30s} {tot - cnt['window fmas']:14.1f}")
    print(f"window: {win} v_pk_fma_f32 + {sc} scalar fmas = {2 * win + sc} fmas "
          f"(16 px x 147 = 2352 per tile-thread)")


if __name__ == "__main__":
    main()
