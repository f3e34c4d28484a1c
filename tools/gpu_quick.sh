#!/bin/bash
# Iteration session: GPU suite, headline bench (+ optional extra bench args), kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r03q}
bash tools/gpu_run.sh \
 "pytest_gpu|600|python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}" \
 "bench|300|python bench.py --steps 500 --cpu-sample 0" \
 "bench_c5|300|python bench.py --workload c5 --steps 100 --warmup 3" \
 "rocprof|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$T -o run -- python bench.py --steps 20 --warmup 2 --cpu-sample 0 --no-profile"
