#!/bin/bash
# Round-3 final evidence session: GPU suite, smoke, headline bench, configs[3] at N = 1 with
# --verify, configs[4] and configs[2] lines, the N = 2 launcher path rehearsed over gloo, a
# kernel trace, then the SQ / HBM counter passes (tools/gpu_pmc_r03.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r03}
bash tools/gpu_run.sh \
 "pytest_gpu|400|python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread" \
 "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench|300|python bench.py" \
 "bench_c4|300|python bench.py --workload c4 --steps 5 --warmup 1 --verify" \
 "bench_c5|300|python bench.py --workload c5 --cpu-sample 0" \
 "bench_c3|300|python bench.py --workload c3 --steps 3 --warmup 1" \
 "rehearsal_n2|400|BENCH_DIST_BACKEND=gloo python bench.py --gpus 2 --frames 256 --steps 2 --warmup 1 --verify" \
 "rocprof|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$T -o run -- python bench.py --steps 20 --warmup 2 --cpu-sample 0 --no-profile" || exit 1
TAG=$T bash tools/gpu_pmc_r03.sh
