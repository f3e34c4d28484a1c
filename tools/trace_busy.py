"""Busy / overlap analysis of a rocprofv3 kernel trace (diagnostic): over the last
`--window` ms of the trace, the fraction of time with >= 1 kernel running, the
per-kernel total durations, and the time-weighted concurrency."""
import csv, glob, sys, collections
path = sys.argv[1]
if not path.endswith(".csv"):
    path = sorted(glob.glob(f"{path}/**/*kernel_trace.csv", recursive=True))[0]
win = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[:34])
        for r in csv.DictReader(open(path))]
rows.sort()
t_end = max(e for _, e, _ in rows)
t0 = t_end - win * 1e6
sel = [(max(s, t0), e, n) for s, e, n in rows if e > t0]
ev = sorted([(s, 1) for s, _, _ in sel] + [(e, -1) for _, e, _ in sel])
busy = 0.0; conc = 0.0; cur = 0; last = t0
for t, d in ev:
    if cur > 0:
        busy += t - last
        conc += cur * (t - last)
    cur += d; last = t
tot = collections.defaultdict(float)
for s, e, n in sel:
    tot[n] += e - s
span = t_end - t0
print(f"window {span/1e6:.2f} ms: busy {busy/span*100:.1f} %, mean concurrency while busy {conc/max(busy,1):.2f}")
for n, v in sorted(tot.items(), key=lambda kv: -kv[1])[:14]:
    print(f"  {n:36s} {v/1e6:8.3f} ms ({v/span*100:5.1f} % of window)")
