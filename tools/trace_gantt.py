"""Text timeline of a rocprofv3 kernel trace (diagnostic): the dispatches of a steady-state
window (default: the 4th-last .. 2nd-last starts of the anchor kernel, k_match_compact: one per
step, i.e. two pipelined steps), one line
each — start offset, duration, queue/stream, kernel, grid — plus per-stream busy time and the
time with no kernel running.

usage: python tools/trace_gantt.py <trace dir or kernel_trace.csv> [first_step_from_end=4] [steps=2] [anchor]"""
import csv
import glob
import sys

path = sys.argv[1]
if not path.endswith(".csv"):
    path = sorted(glob.glob(f"{path}/**/*kernel_trace.csv", recursive=True))[0]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 4
nst = int(sys.argv[3]) if len(sys.argv) > 3 else 2
anchor = sys.argv[4] if len(sys.argv) > 4 else "k_match_compact"
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
firsts = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
a = firsts[-back]
b = firsts[-back + nst] if -back + nst < 0 else len(rows)
t0 = int(rows[a]["Start_Timestamp"])
t1 = int(rows[b]["Start_Timestamp"]) if b < len(rows) else max(int(r["End_Timestamp"]) for r in rows)
qkey = "Stream_Id" if "Stream_Id" in rows[0] else ("Queue_Id" if "Queue_Id" in rows[0] else None)
print(f"window {(t1 - t0) / 1e3:.1f} us, {nst} step starts")
busy = {}
ev = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e <= t0 or s >= t1:
        continue
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sfm::", "")[:34]
    q = r.get(qkey, "?") if qkey else "?"
    grid = r.get("Grid_Size_X", r.get("Grid_X", "")) + "x" + r.get("Grid_Size_Y", r.get("Grid_Y", ""))
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{q:>3s}  {name:34s} {grid}")
    busy[q] = busy.get(q, 0) + min(e, t1) - max(s, t0)
    ev += [(max(s, t0), 1), (min(e, t1), -1)]
ev.sort()
idle, cur, last = 0, 0, t0
for t, d in ev:
    if cur == 0:
        idle += t - last
    cur += d
    last = t
idle += t1 - last
print("per-queue busy (us):", {k: round(v / 1e3, 1) for k, v in busy.items()}, f" idle (no kernel) {idle / 1e3:.1f} us")
