#!/bin/bash
# PMC counter passes (each its own rocprofv3 run; no tracing domains mixed with --pmc).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-pmc}
CMD="python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-profile"
i=0
for set in "${@}"; do
  i=$((i+1))
  echo "[$(date +%T)] pass $i: $set" | tee -a $OUT/status.txt
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/${TAG}_p$i -o run -- $CMD > $OUT/${TAG}_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc" | tee -a $OUT/status.txt
  if [ $rc -ne 0 ]; then tail -20 $OUT/${TAG}_p$i.log; exit $rc; fi
done
echo done
