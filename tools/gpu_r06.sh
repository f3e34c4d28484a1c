#!/bin/bash
# Round-6 GPU evidence, one gpurun call: STEPS selects what runs (space-separated):
#   tests   the GPU suite          smoke   __graft_entry__.smoke()
#   bench   the driver's command (python bench.py --gpus 1 --steps 20 --warmup 5) BENCH_N times
#   trace   rocprofv3 --kernel-trace --stats of the driver's command + tools/trace_roofline.py
#   c3 c4 c5  the other BASELINE configurations        sq  one SQ counter pass
#   pmc     FETCH_SIZE / WRITE_SIZE passes (HBM traffic per kernel)
# Outputs: gpurun_out/<TAG>_*.  Every GPU step has its own time limit; the first failure ends
# the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r06}
O=gpurun_out
mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$to" "$@" > "$O/${T}_$name.out" 2> "$O/${T}_$name.err"
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -n 30 "$O/${T}_$name.err" "$O/${T}_$name.out"; exit $rc; }
}
for s in ${STEPS:-tests smoke bench trace}; do
  case $s in
    tests)
      step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
      tail -1 $O/${T}_pytest_gpu.out ;;
    smoke)
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
      tail -1 $O/${T}_smoke.out ;;
    bench)
      for i in $(seq 1 ${BENCH_N:-1}); do
        step bench_$i 300 python bench.py ${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5}
        python -c "import json;d=json.load(open('$O/${T}_bench_$i.out'));r=d['roofline'];print('c2', d['value'], d['ms_per_step'], r['frac'], r['ms_per_step'], r['launch_sum'])"
      done ;;
    trace)
      step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python bench.py --steps 20 --warmup 5 --cpu-sample 0 --no-profile
      python tools/trace_summary.py $O/${T}_prof > $O/${T}_trace_summary.txt
      python tools/trace_roofline.py $O/${T}_prof --steps 20 --warmup 5 --bench $O/${T}_trace.out > $O/${T}_trace_roofline.json
      cat $O/${T}_trace_roofline.json ;;
    c3) step bench_c3 300 python bench.py --workload c3 --steps 5 --warmup 2 --cpu-sample 0
        python -c "import json;d=json.load(open('$O/${T}_bench_c3.out'));print('c3', d['value'], d['ms_per_step'])" ;;
    c4) step bench_c4 300 python bench.py --workload c4 --steps 5 --warmup 2 --cpu-sample 0 --verify ${C4_ARGS:-}
        python -c "import json;d=json.load(open('$O/${T}_bench_c4.out'));print('c4', d['value'], d['ms_per_step'], d.get('collective'))" ;;
    c5) step bench_c5 300 python bench.py --workload c5 --steps 100 --warmup 5 --cpu-sample 0
        python -c "import json;d=json.load(open('$O/${T}_bench_c5.out'));print('c5', d['value'], d['ms_per_step'])" ;;
    emu)
      step emu_bench 300 python bench.py --workload c4 --frames 256 --steps 5 --warmup 2 --emulate-exchange ${EMU_WG:-32}
      python -c "import json;d=json.load(open('$O/${T}_emu_bench.out'));print('emu', json.dumps(d['collective']))"
      step emu_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_emu_prof -o run -- python bench.py --workload c4 --frames 256 --steps 2 --warmup 1 --emulate-exchange ${EMU_WG:-32}
      python tools/trace_summary.py $O/${T}_emu_prof > $O/${T}_emu_trace_summary.txt
      python tools/trace_gantt.py $O/${T}_emu_prof 3 2 k_copy_wg > $O/${T}_emu_gantt.txt || true ;;
    sq)
      step pmc_sq 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/${T}_pmc_sq -o run -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-profile
      python tools/sq_summary.py $O/${T}_pmc_sq $O/${T}_sq_counters "# $T build, bench.py --steps 2 --warmup 1" > /dev/null ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        step pmc_$c 300 rocprofv3 --pmc $c --output-format csv -d $O/${T}_pmc_$c -o run -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-profile
      done
      python tools/pmc_traffic.py $O/${T}_pmc_FETCH_SIZE $O/${T}_pmc_WRITE_SIZE $O/${T}_pmc_traffic.json ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
