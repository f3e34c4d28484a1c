"""One kernel's SQ counters merged over several rocprofv3 --pmc passes (diagnostic):

    python tools/pmc_sum.py <kernel-substring> <label> <pass_dir> [<pass_dir> ...]

Per-dispatch averages, and the shares of SQ_WAVE_CYCLES spent waiting (s_waitcnt / barrier:
SQ_WAIT_ANY), stalled at issue (SQ_WAIT_INST_ANY; its LDS part SQ_WAIT_INST_LDS) and issuing
(SQ_ACTIVE_INST_ANY); MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024)."""
import collections
import csv
import glob
import sys


def main():
    kern, label, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    avg, us = {}, []
    for d in dirs:
        path = sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True))[0]
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(path)):
            if kern not in r["Kernel_Name"]:
                continue
            key = r["Dispatch_Id"]
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                us.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        disp = sorted(per, key=int)[1:] or sorted(per, key=int)  # first dispatch: warm-up
        for name in per[disp[0]]:
            avg[name] = sum(per[k][name] for k in disp) / len(disp)
    wc = avg.get("SQ_WAVE_CYCLES", 0) or 1
    cyc = avg.get("GRBM_GUI_ACTIVE", 0) / 8 * 1024 or 1
    f = lambda n: 100 * avg.get(n, 0) / wc
    print(f"{label}: {kern} {sum(us) / max(len(us), 1):.1f} us/dispatch (under PMC); wave cycles: "
          f"wait {f('SQ_WAIT_ANY'):.1f}% issue-stall {f('SQ_WAIT_INST_ANY'):.1f}% (LDS {f('SQ_WAIT_INST_LDS'):.1f}%) "
          f"active {f('SQ_ACTIVE_INST_ANY'):.1f}%; MFMA busy {100 * avg.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / cyc:.1f}%; "
          f"LDS bank-conflict / active cycles {avg.get('SQ_LDS_BANK_CONFLICT', 0):.0f} / {avg.get('SQ_LDS_IDX_ACTIVE', 0):.0f}; "
          f"insts VALU {avg.get('SQ_INSTS_VALU', 0):.0f} LDS {avg.get('SQ_INSTS_LDS', 0):.0f} SALU {avg.get('SQ_INSTS_SALU', 0):.0f}")


if __name__ == "__main__":
    main()
