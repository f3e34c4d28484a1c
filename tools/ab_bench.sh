#!/bin/bash
# Same-box A/B of two library builds on the driver's bench, N alternating pairs (default 6) of
# `bench.py --steps 50 --warmup 5`: A = ab_head/base (a saved build), B = the in-tree library.
# Prints each run and the mean / spread per side.  usage: bash tools/ab_bench.sh [pairs] [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-6}; shift || true
A=$PWD/ab_head/base/libsfmfeat.so
B=$PWD/sfmfromscratch_amd/lib/libsfmfeat.so
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    SFMFEAT_LIB=$lib timeout -k 10 200 python bench.py --steps 50 --warmup 5 --cpu-sample 0 --no-profile "$@" > gpurun_out/abb_${v}_$i.json 2> gpurun_out/abb_${v}_$i.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/abb_${v}_$i.json'));print('$v', $i, d['value'], d['ms_per_step'])"
  done
done | tee gpurun_out/abb_runs.txt
python - <<'PY'
import statistics as st
r = {"A": [], "B": []}
for line in open("gpurun_out/abb_runs.txt"):
    v, i, val, ms = line.split()
    r[v].append(float(val))
for v in "AB":
    print(f"{v}: mean {st.mean(r[v]):.0f} img/s, stdev {st.pstdev(r[v]):.0f}, min {min(r[v]):.0f}, max {max(r[v]):.0f}")
print(f"B/A = {st.mean(r['B']) / st.mean(r['A']):.4f}")
PY
