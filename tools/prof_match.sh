#!/bin/bash
# Matcher-only PMC passes (k_match_mfma in isolation, tools/bench_match.py --allpairs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03m}
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/avail_$T.txt 2>&1 || true
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_${T}_$i -o run -- python tools/bench_match.py --iters 3 ${MATCH_ARGS:---allpairs} > gpurun_out/pmc_${T}_$i.log 2>&1 || exit 1
done
echo done
