"""Per-kernel SQ counter summary from one rocprofv3 --pmc pass (diagnostic):

    python tools/sq_summary.py <pmc_pass_dir> <out_prefix> [header line]

writes <out_prefix>.json (per-dispatch averages of every counter, by kernel) and
<out_prefix>.txt (the table below).  Derived columns (MI355X_MICROARCH.md):
  cycles/XCD = GRBM_GUI_ACTIVE / 8
  VALU busy  = 4 * SQ_INSTS_VALU / (cycles/XCD * 1024 SIMDs)   (a wave64 VALU op: 4 cycles)
  MFMA busy  = SQ_VALU_MFMA_BUSY_CYCLES / (cycles/XCD * 1024)
  wait / issue-stall = SQ_WAIT_ANY / SQ_WAVE_CYCLES, SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
"""
import collections
import csv
import glob
import json
import sys


def main():
    src, out = sys.argv[1], sys.argv[2]
    header = sys.argv[3] if len(sys.argv) > 3 else ""
    path = sorted(glob.glob(f"{src}/**/*counter_collection.csv", recursive=True))[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, dispatch) -> counters
    dur = {}
    for r in csv.DictReader(open(path)):
        key = (r["Kernel_Name"], r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    us = collections.defaultdict(float)
    for (k, d), c in per.items():
        n[k] += 1
        us[k] += dur[(k, d)]
        for name, v in c.items():
            agg[k][name] += v
    avg = {k: {name: round(v / n[k]) for name, v in sorted(agg[k].items())} for k in agg}
    json.dump(avg, open(out + ".json", "w"), indent=1)
    lines = []
    if header:
        lines.append(f"# {header}")
    lines.append("# per dispatch averages; VALU busy = 4 * SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 * 1024); "
                 "MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024);")
    lines.append("# wait / issue-stall = SQ_WAIT_ANY / SQ_WAVE_CYCLES, SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES")
    lines.append(f"{'kernel':55s} {'disp':>5s} {'us':>8s} {'VALU%':>6s} {'MFMA%':>6s} {'wait%':>6s} {'issue-stall%':>12s}")
    order = sorted(avg, key=lambda k: -us[k])
    for k in order:
        c = avg[k]
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8 * 1024
        wc = c.get("SQ_WAVE_CYCLES", 0)
        valu = 100 * 4 * c.get("SQ_INSTS_VALU", 0) / cyc if cyc else 0.0
        mfma = 100 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / cyc if cyc else 0.0
        wait = 100 * c.get("SQ_WAIT_ANY", 0) / wc if wc else 0.0
        stall = 100 * c.get("SQ_WAIT_INST_ANY", 0) / wc if wc else 0.0
        name = k.split("(")[0].replace("void ", "")[:55]
        lines.append(f"{name:55s} {n[k]:5d} {us[k] / n[k]:8.1f} {valu:6.1f} {mfma:6.1f} {wait:6.1f} {stall:12.1f}")
    open(out + ".txt", "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:16]))


if __name__ == "__main__":
    main()
