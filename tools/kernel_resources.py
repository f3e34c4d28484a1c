#!/usr/bin/env python3
"""Resource usage (VGPRs, AGPRs, SGPRs, LDS, spills, scratch) of the kernels in a built HIP
object or shared library, from the gfx950 code object's metadata notes.

usage: tools/kernel_resources.py <file.o|lib.so> [name-substring ...]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(path, tmp):
    fb = os.path.join(tmp, "fb.bin")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, fb], check=True)
    data = open(fb, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    for n, i in enumerate(starts):
        j = starts[n + 1] if n + 1 < len(starts) else len(data)
        b, e = os.path.join(tmp, f"b{n}.bin"), os.path.join(tmp, f"b{n}.elf")
        open(b, "wb").write(data[i:j])
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={b}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={e}"], check=True)
        yield e


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    with tempfile.TemporaryDirectory() as tmp:
        for e in code_objects(path, tmp):
            t = subprocess.run([os.path.join(LLVM, "llvm-readobj"), "--notes", e], check=True,
                               capture_output=True, text=True).stdout
            for blk in t.split("- .agpr_count")[1:]:
                name = re.search(r"\.name:\s+(\S+)", blk).group(1)
                if pats and not any(p in name for p in pats):
                    continue
                g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, None])[1]
                agpr = re.match(r":\s+(\d+)", blk)
                print(f"{name}: vgpr {g('vgpr_count')} agpr {agpr.group(1) if agpr else '?'} sgpr {g('sgpr_count')} "
                      f"lds {g('group_segment_fixed_size')} vspill {g('vgpr_spill_count')} sspill {g('sgpr_spill_count')} "
                      f"scratch {g('private_segment_fixed_size')}")


if __name__ == "__main__":
    main()
