#!/bin/bash
# Harris-only PMC passes (k_harris<7> in isolation, tools/ablate_harris.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03h}
mkdir -p gpurun_out
P1=${P1:-"SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"}
P2=${P2:-"SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"}
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_${T}_$i -o run -- python tools/ablate_harris.py > gpurun_out/pmc_${T}_$i.log 2>&1 || exit 1
done
echo done
