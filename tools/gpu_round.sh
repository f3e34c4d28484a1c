#!/bin/bash
# One gpurun session: GPU parity tests -> smoke -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash/timeout/abort ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${TAG:-r01}
step() {  # step NAME SECONDS CMD...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] start $name" | tee -a $OUT/status.txt
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $OUT/status.txt
  return $rc
}
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 2 ] || [ "$1" -eq 3 ] || [ "$1" -eq 4 ]; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu "${TEST_TIMEOUT:-900}" python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-}; rc=$?
  if fatal $rc; then tail -30 $OUT/pytest_gpu.log; exit $rc; fi
  tail -15 $OUT/pytest_gpu.log
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || { tail -20 $OUT/smoke.log; exit 1; }
fi
step bench 600 python bench.py --steps ${STEPS:-10} --warmup 3 ${BENCH_ARGS:-} || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
if [ "${SKIP_PROF:-0}" != 1 ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
       python bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-profile || exit 1
  find $OUT/prof_$TAG -name "*kernel_stats.csv" | head -3
  python tools/trace_summary.py $OUT/prof_$TAG > $OUT/trace_summary_$TAG.txt 2>&1 || true
fi
if [ "${PMC:-0}" = 1 ]; then  # HBM traffic: FETCH_SIZE and WRITE_SIZE in separate passes, no tracing
  for c in FETCH_SIZE WRITE_SIZE; do
    step pmc_$c 600 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_${TAG}_$c -o run -- \
         python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-profile || exit 1
  done
  python tools/pmc_traffic.py $OUT/pmc_${TAG}_FETCH_SIZE $OUT/pmc_${TAG}_WRITE_SIZE $OUT/pmc_traffic_$TAG.json
fi
echo done
