"""Summarise a rocprofv3 kernel_trace.csv per (kernel, grid size): count, mean and total
duration — distinguishes the pyramid levels of one stage (diagnostic).  With --timeline,
also print the dispatches of the last extract+match step in order."""
import collections
import csv
import glob
import sys

path = sys.argv[1]
if not path.endswith(".csv"):
    path = sorted(glob.glob(f"{path}/**/*kernel_trace.csv", recursive=True))[0]
rows = list(csv.DictReader(open(path)))
agg = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
    grid = tuple(int(r.get(f"Grid_Size_{a}", r.get(f"Grid_{a}", 0)) or 0) for a in "XYZ")
    agg[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in agg.values())
print(f"{'kernel':40s} {'grid':>22s} {'n':>4s} {'mean_us':>9s} {'total_us':>10s}")
for (name, grid), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{name:40s} {str(grid):>22s} {len(v):4d} {sum(v) / len(v):9.1f} {sum(v):10.1f}")
print(f"total {tot:.1f} us")

if "--timeline" in sys.argv:
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    firsts = [i for i, r in enumerate(rows) if "k_down2" in r["Kernel_Name"]]
    start = firsts[-3] if len(firsts) >= 3 else 0
    t0 = int(rows[start]["Start_Timestamp"])
    print("\n-- last step --")
    for r in rows[start:]:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sfm::", "")[:34]
        s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{name:36s} +{(s0 - t0) / 1e3:8.1f} us  {(e0 - s0) / 1e3:7.1f} us")
