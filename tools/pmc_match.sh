#!/bin/bash
# Where k_match_mfma's wave cycles go, per sweep ablation (diagnostic library, SFMFEAT_MATCH_ABL:
# 0 full, 1 no epilogue, 2 no MFMAs, 3 neither): two SQ counter passes each over tools/bench_match.py,
# summed over the sweep's dispatches (tools/pmc_sum.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE"
LIB=${SFMFEAT_LIB:-$PWD/sfmfromscratch_amd/lib_diag/libsfmfeat.so}
for a in ${ABLS:-0 1 2 3}; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    SFMFEAT_LIB=$LIB SFMFEAT_MATCH_ABL=$a timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv \
      -d gpurun_out/pmcm_${a}_$i -o run -- python tools/bench_match.py --iters 5 ${MATCH_ARGS:-} \
      > gpurun_out/pmcm_${a}_$i.log 2>&1 || exit 1
  done
  python tools/pmc_sum.py k_match_mfma "MATCH_ABL=$a" gpurun_out/pmcm_${a}_1 gpurun_out/pmcm_${a}_2
done
