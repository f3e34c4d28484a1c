#!/bin/bash
# r02 session A: GPU suite, configs[3] leg at N=1, SQ counters for Harris / matcher.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "[$(date +%T)] $name" >> $OUT/status.txt
  timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" >> $OUT/status.txt
  [ $rc -eq 0 ] || { tail -30 $OUT/$name.log; exit $rc; }; }
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
tail -3 $OUT/pytest_gpu.log
run bench_c4 300 python bench.py --workload c4 --steps 3 --warmup 1
tail -1 $OUT/bench_c4.log
run bench_c4_halo 300 python bench.py --workload c4 --exchange halo --steps 3 --warmup 1
tail -1 $OUT/bench_c4_halo.log
run pmc_sq 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_sq_r02 -o run -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-profile
echo done
