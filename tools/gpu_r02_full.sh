#!/bin/bash
# Full evidence session for the current build: GPU suite, smoke, the headline bench, the other
# BASELINE configurations, a kernel-trace profile and the SQ / traffic counter passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r02}
exec bash tools/gpu_run.sh \
 "pytest_gpu|600|python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread" \
 "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench|300|python bench.py" \
 "bench_c3|300|python bench.py --workload c3 --steps 3 --warmup 1" \
 "bench_c4|300|python bench.py --workload c4 --steps 3 --warmup 1" \
 "bench_c5|300|python bench.py --workload c5 --steps 100 --warmup 3" \
 "rocprof|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$T -o run -- python bench.py --steps 20 --warmup 2 --cpu-sample 0 --no-profile" \
 "pmc_sq|120|rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq_$T -o run -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-profile" \
 "pmc_f|120|rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f_$T -o run -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-profile" \
 "pmc_w|120|rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w_$T -o run -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-profile"
