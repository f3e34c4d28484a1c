#!/bin/bash
# Counter passes on the headline bench: SQ issue/stall counters (tools/sq_summary.py)
# and HBM traffic (FETCH_SIZE, WRITE_SIZE in separate passes; tools/pmc_traffic.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r03}
TAG=pmc_$T bash tools/gpu_pmc.sh "SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" FETCH_SIZE WRITE_SIZE || exit 1
python tools/sq_summary.py gpurun_out/pmc_${T}_p1 gpurun_out/${T}_sq_counters "# $T build, bench.py --steps 2 --warmup 1" || exit 1
python tools/pmc_traffic.py gpurun_out/pmc_${T}_p2 gpurun_out/pmc_${T}_p3 gpurun_out/${T}_pmc_traffic.json || exit 1
cat gpurun_out/${T}_sq_counters.txt | head -20
