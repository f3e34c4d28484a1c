#!/bin/bash
# A/B of environment switches on the headline bench: ab_env.sh "VAR=a" "VAR=b,VAR2=c" ... (each
# run REPS times (2), interleaved; commas separate several variables of one variant); prints
# img/s, ms/step and the per-stage ms of every run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env ${e//,/ } timeout -k 10 150 python bench.py --cpu-sample 0 ${BENCH_ARGS:-} > gpurun_out/ab_${i}_$rep.log 2>&1 || { tail -5 gpurun_out/ab_${i}_$rep.log; exit 1; }
    tail -1 gpurun_out/ab_${i}_$rep.log | python -c '
import json,sys
d=json.loads(sys.stdin.read()); st=d.get("stages_ms",{})
print(sys.argv[1], d["value"], d["ms_per_step"], "frac", (d.get("roofline") or {}).get("frac"), " ".join("%s=%s" % (k, v["ms_per_step"]) for k,v in st.items()))' "$e"
  done
done
