#!/usr/bin/env python3
"""Recompute bench.py's Harris roofline from a rocprofv3 --kernel-trace of the same command.

bench.py (c2) times every k_harris launch of its timed region by kernel-active spans and
reports two attributions per step: the union of the launches' intervals over both lanes
(`roofline.ms_per_step`, `frac`) and the sum of the launch durations (`roofline.launch_sum`).
This tool computes both from the trace, for the launches of the timed region:
  the trace holds, in order, [profile pass: P steps, one batch at a time] (absent with
  --no-profile) [warm-up: W steps] [timed: K steps] [same-batch pass: K steps]; the launches
  are sorted by start time and the timed block is launches [(P + W) L, (P + W + K) L).
usage: trace_roofline.py TRACE_DIR_OR_CSV --steps K --warmup W [--profile-steps P] [--levels 4]
       [--bench bench.json]   (compares with the line's roofline when given)"""
import argparse
import csv
import glob
import json
import sys

PEAK = 157.3
FLOP_PER_PX = 328


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--levels", type=int, default=4)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--hw", default="1080x1920")
    ap.add_argument("--kernel", default="k_harris<7")
    ap.add_argument("--bench", default=None)
    a = ap.parse_args()
    path = a.trace
    if not path.endswith(".csv"):
        path = sorted(glob.glob(f"{path}/**/*kernel_trace.csv", recursive=True))[0]
    rows = [r for r in csv.DictReader(open(path)) if a.kernel in r["Kernel_Name"].replace("sfm::", "")]
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    L, K = a.levels, a.steps
    lo = (a.profile_steps + a.warmup) * L
    blk = iv[lo:lo + K * L]
    if len(blk) != K * L:
        raise SystemExit(f"{len(iv)} {a.kernel} launches in the trace, expected at least {lo + K * L}")
    ssum = sum(e - s for s, e in blk)
    union, c0, c1 = 0, blk[0][0], blk[0][1]
    for s, e in blk[1:]:
        if s > c1:
            union += c1 - c0
            c0, c1 = s, e
        else:
            c1 = max(c1, e)
    union += c1 - c0
    H, W = (int(v) for v in a.hw.split("x"))
    flop = FLOP_PER_PX * sum((H >> l) * (W >> l) for l in range(L)) * a.batch
    out = {"trace": path, "kernel": a.kernel, "launches_in_trace": len(iv), "timed_block": [lo, lo + K * L],
           "avg_launch_ms": round(ssum / len(blk) / 1e6, 4),
           "launch_sum_ms_per_step": round(ssum / K / 1e6, 4), "union_ms_per_step": round(union / K / 1e6, 4),
           "frac_launch_sum": round(flop / (ssum / K / 1e9) / 1e12 / PEAK, 4),
           "frac_union": round(flop / (union / K / 1e9) / 1e12 / PEAK, 4)}
    if a.bench:
        d = json.loads(open(a.bench).read().strip().splitlines()[-1])
        r = d["roofline"]
        out["bench"] = {"ms_per_step": d["ms_per_step"], "frac_union": r["frac"],
                        "union_ms_per_step": r.get("ms_per_step"), "avg_launch_ms": r.get("avg_launch_ms"),
                        "frac_launch_sum": (r.get("launch_sum") or {}).get("frac")}
        out["bench_over_trace"] = {"frac_union": round(r["frac"] / out["frac_union"], 4),
                                   "frac_launch_sum": round((r.get("launch_sum") or {}).get("frac", 0.0)
                                                            / out["frac_launch_sum"], 4)}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
