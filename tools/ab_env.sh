#!/bin/bash
# Same-box A/B/C... of one environment switch on the driver's bench: N rounds (default 4) of
# `bench.py --steps 50 --warmup 5`, the values of VAR in turn each round (an empty value
# leaves VAR unset).  usage: VAR=SFMFEAT_HARRIS_SLOTS VALS="448 512" bash tools/ab_env.sh [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-4}
mkdir -p gpurun_out
: > gpurun_out/abe_runs.txt
for i in $(seq 1 $N); do
  for v in $VALS; do
    if [ "$v" = "-" ]; then
      timeout -k 10 200 env -u $VAR python bench.py --steps 50 --warmup 5 --cpu-sample 0 --no-profile > gpurun_out/abe.json 2> gpurun_out/abe.err || exit 1
    else
      env $VAR=$v timeout -k 10 200 python bench.py --steps 50 --warmup 5 --cpu-sample 0 --no-profile > gpurun_out/abe.json 2> gpurun_out/abe.err || exit 1
    fi
    python -c "import json;d=json.load(open('gpurun_out/abe.json'));print('$v', $i, d['value'], d['ms_per_step'])" | tee -a gpurun_out/abe_runs.txt
  done
done
python - <<'PY'
import collections, statistics as st
r = collections.defaultdict(list)
for line in open("gpurun_out/abe_runs.txt"):
    v, i, val, ms = line.split()
    r[v].append(float(val))
for v, xs in r.items():
    print(f"{v}: mean {st.mean(xs):.0f} img/s, stdev {st.pstdev(xs):.0f}, n {len(xs)}")
PY
