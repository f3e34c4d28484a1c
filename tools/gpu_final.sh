#!/bin/bash
# End-of-round evidence on one GPU: GPU suite, smoke, the driver's bench command three times,
# the other BASELINE configs, a rocprofv3 kernel trace of the headline bench, HBM traffic and SQ
# counter passes, and the N = 2 launcher rehearsal over gloo.  Outputs: gpurun_out/<TAG>_*.
# PHASE=1: tests, smoke and the benches; PHASE=2: trace, PMC passes, rehearsal (one gpurun call
# each fits its time limit); unset: everything.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r05_final}
PH=${PHASE:-0}
O=gpurun_out
mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$to" "$@" > "$O/${T}_$name.out" 2> "$O/${T}_$name.err"
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -20 "$O/${T}_$name.err" "$O/${T}_$name.out"; exit $rc; }
}
if [ "$PH" != 2 ]; then
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
  tail -1 $O/${T}_pytest_gpu.out
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  tail -1 $O/${T}_smoke.out
fi
for i in 1 2 3; do
  step bench_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5
  python -c "import json;d=json.load(open('$O/${T}_bench_$i.out'));print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
step bench_c3 300 python bench.py --workload c3 --steps 5 --warmup 2 --cpu-sample 0
step bench_c4 300 python bench.py --workload c4 --steps 5 --warmup 2 --cpu-sample 0 --verify
step bench_c5 300 python bench.py --workload c5 --steps 100 --warmup 5 --cpu-sample 0
for w in c3 c4 c5; do python -c "import json;d=json.load(open('$O/${T}_bench_$w.out'));print('$w', d['value'], d['ms_per_step'])"; done
fi
[ "$PH" = 1 ] && { echo done; exit 0; }
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python bench.py --steps 20 --warmup 5 --cpu-sample 0 --no-profile
python tools/trace_summary.py $O/${T}_prof > $O/${T}_trace_summary.txt
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c 300 rocprofv3 --pmc $c --output-format csv -d $O/${T}_pmc_$c -o run -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-profile
done
python tools/pmc_traffic.py $O/${T}_pmc_FETCH_SIZE $O/${T}_pmc_WRITE_SIZE $O/${T}_pmc_traffic.json
step pmc_sq 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/${T}_pmc_sq -o run -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-profile
python tools/sq_summary.py $O/${T}_pmc_sq $O/${T}_sq_counters "# $T build, bench.py --steps 2 --warmup 1" > /dev/null
if [ "${REHEARSAL:-1}" = 1 ]; then
  BENCH_DIST_BACKEND=gloo step rehearsal_c4 600 python bench.py --gpus 2 --workload c4 --frames 256 --steps 2 --warmup 1 --cpu-sample 0 --verify
  tail -1 $O/${T}_rehearsal_c4.out | cut -c1-300
fi
echo done
