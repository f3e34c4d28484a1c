#!/bin/bash
# Round-3 evidence session: GPU suite, smoke, headline bench, configs[3] at N = 1, the
# N = 2 launcher path rehearsed over gloo on the one GPU (with --verify), a kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r03}
bash tools/gpu_run.sh \
 "pytest_gpu|900|python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}" \
 "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench|300|python bench.py" \
 "bench_c4|300|python bench.py --workload c4 --steps 5 --warmup 1 --verify" \
 "rehearsal_n2|400|BENCH_DIST_BACKEND=gloo python bench.py --gpus 2 --frames 256 --steps 2 --warmup 1 --verify" \
 "rocprof|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$T -o run -- python bench.py --steps 20 --warmup 2 --cpu-sample 0 --no-profile"
