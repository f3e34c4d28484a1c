#!/bin/bash
# A/B of one kernel's duration under an environment switch: tools/bench_match.py (or $CMD) under
# a rocprofv3 kernel trace per setting, interleaved, mean / min of the kernel's launches.
# usage: VAR=SFMFEAT_MATCH_APPEND VALS="0 1 0 1" KERNEL=k_match_mfma bash tools/ab_kernel.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CMD=${CMD:-python tools/bench_match.py --iters 20}
i=0
for v in $VALS; do
  i=$((i+1))
  env $VAR=$v timeout -k 5 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_${VAR}_$i -o run -- \
    $CMD > gpurun_out/ab_${VAR}_$i.log 2>&1 || exit 1
  python - "$VAR" "$v" "$i" "$KERNEL" <<'PY'
import csv, glob, sys
var, v, i, kern = sys.argv[1:5]
rows = []
for f in glob.glob(f"gpurun_out/ab_{var}_{i}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            rows.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
rows = rows[1:] or rows
print(f"{var}={v}: {kern} {len(rows)} launches, mean {sum(rows) / max(len(rows), 1):.1f} us, min {min(rows):.1f} us")
PY
  tail -1 gpurun_out/ab_${VAR}_$i.log
done
