#!/usr/bin/env python3
"""Compressed instruction sequence of one kernel of the built library (no GPU needed):
M = MFMA, R = ds_read, W = ds_write, D = LDS-DMA / buffer load, S = global store,
vN = N vector ALU instructions, [lN] / [vN] = s_waitcnt lgkmcnt(N) / vmcnt(N), |B| = barrier,
>x = branch.  Shows how far ahead of their MFMAs the fragment reads are issued.
usage: tools/isa_seq.py kernel-substring [lib.so]"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa_phases import ROOT, disassemble  # noqa: E402


def sequence(body):
    seq = []
    for line in body.splitlines()[1:]:
        if not re.match(r"\s+[a-z]", line):
            continue
        op = line.split()[0]
        if op.startswith("v_mfma"):
            seq.append("M")
        elif op.startswith("ds_read"):
            seq.append("R")
        elif op.startswith("ds_write"):
            seq.append("W")
        elif op.startswith("s_waitcnt"):
            m, v = re.search(r"lgkmcnt\((\d+)\)", line), re.search(r"vmcnt\((\d+)\)", line)
            seq.append("[l%s]" % m.group(1) if m else ("[v%s]" % v.group(1) if v else "[w]"))
        elif op == "s_barrier":
            seq.append("|B|")
        elif op.startswith("v_"):
            seq.append("v")
        elif op.startswith("s_cbranch") or op == "s_branch":
            seq.append(">" + op[9:] + " ")
        elif op.startswith(("global_load_lds", "buffer_load")):
            seq.append("D")
        elif op.startswith("global_store"):
            seq.append("S")
    s = "".join(seq)
    return re.sub(r"v{2,}", lambda m: "v%d" % len(m.group(0)), s)


def main():
    pat = sys.argv[1]
    lib = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "sfmfromscratch_amd", "lib", "libsfmfeat.so")
    for f in re.split(r"\n(?=[0-9a-f]{16} <)", disassemble(lib)):
        m = re.match(r"[0-9a-f]{16} <(\S+)>:", f)
        if m and pat in m.group(1):
            print(m.group(1))
            print(sequence(f))
            return
    raise SystemExit(f"no kernel matching {pat!r}")


if __name__ == "__main__":
    main()
