"""Per-level k_harris / k_down2x3 durations from serial (SFMFEAT_SERIAL=1) kernel traces:
python tools/harris_l0_summary.py TAG... reads gpurun_out/hl0_TAG/**/*kernel_trace.csv.  Launches
of one shape alternate between the levels that share it (L0 / L1 of form 0), in issue order."""
import csv
import glob
import sys

for tag in sys.argv[1:]:
    p = glob.glob(f"gpurun_out/hl0_{tag}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
                   r.get("Grid_Size_X", "")) for r in csv.DictReader(open(p)))
    d = {}
    for s, e, n, g in rows:
        if "k_harris" in n or "k_down2x3" in n:
            d.setdefault((n, g), []).append((e - s) / 1e3)
    for (n, g), v in sorted(d.items()):
        parts = [v[0::2], v[1::2]] if "k_harris<7, true, 0, 0>" in n else [v]
        for i, w in enumerate(parts):
            print(f"{tag}: {n:34s} {g:>8s} [{i}] n={len(w):3d} mean={sum(w)/len(w):8.1f} min={min(w):8.1f}")
