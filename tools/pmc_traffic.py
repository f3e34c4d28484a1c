"""HBM traffic per launch per kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE),
following MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7:
  bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
(both counters in KiB; on gfx950 FETCH_SIZE reads exactly 1/2 of a wide coalesced
16-B-per-lane stream, the access width of the streaming kernels here).  Writes
profiles/pmc_traffic.json, which bench.py reads for its roofline.traffic field.

    python tools/pmc_traffic.py <fetch_pass_dir> <write_pass_dir> [out.json]
"""
import collections
import csv
import glob
import json
import re
import sys


def short_name(full: str) -> str:
    m = re.match(r"_ZN3sfm(\d+)(\w+)", full)
    if m:  # mangled, non-template: _ZN3sfm12k_match_mfmaE...
        return m.group(2)[: int(m.group(1))]
    name = full.split("(")[0].replace("void ", "").replace("sfm::", "").replace(" ", "")
    t = re.match(r"(k_harris)<(\d+),(?:true,|false,)?0(?:,\d+)?>", name)
    if t:  # both load variants of one window size
        return f"{t.group(1)}<{t.group(2)}>"
    if name.startswith("dq::k_describe_q<"):  # every level's instance
        return "k_describe_q"
    return name


def per_kernel(d: str, counter: str):
    path = sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True))[0]
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = short_name(r["Kernel_Name"])
        tot[k] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return {k: (tot[k], len(disp[k])) for k in tot}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    res = {}
    for k in sorted(set(fetch) | set(write)):
        f, nf = fetch.get(k, (0.0, 1))
        w, nw = write.get(k, (0.0, 1))
        res[k] = round((2.0 * f / max(nf, 1) + w / max(nw, 1)) * 1024)
    doc = {"method": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 per launch, separate rocprofv3 --pmc passes, "
                     "bench.py --steps 2 --warmup 1 (tools/gpu_pmc.sh)",
           "bytes_per_launch": res}
    with open(out, "w") as fo:
        json.dump(doc, fo, indent=1)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]):
        print(f"{k:32s} {v / 1e6:10.2f} MB/launch")


if __name__ == "__main__":
    main()
