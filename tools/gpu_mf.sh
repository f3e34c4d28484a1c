#!/bin/bash
# Harris MFMA-form iteration: GPU parity suite with the form on every level, isolated L0 timing
# of both forms, one SQ counter pass of the MFMA form (tools/prof_harris.sh), optional A/B bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  SFMFEAT_HARRIS_MF=${TEST_MF:-2} timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_mf2.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_mf2.log; [ $rc -eq 0 ] || exit $rc
fi
for m in ${MF_VARIANTS:-"SFMFEAT_HARRIS_MF=0" "SFMFEAT_HARRIS_MF=1"}; do
  env $m timeout -k 10 120 python tools/ablate_harris.py > gpurun_out/abl.txt 2>&1 || exit 1
  echo "$m"; grep B= gpurun_out/abl.txt
done
if [ "${PMC:-1}" = 1 ]; then
  SFMFEAT_HARRIS_MF=${PMC_MF:-1} P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
    P2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE" \
    TAG=mf bash tools/prof_harris.sh > /dev/null && python tools/sq_summary.py gpurun_out/pmc_mf_1 gpurun_out/sq_mf_1 | grep "7, true, 0, ${PMC_FORM:-4}" \
    && python tools/sq_summary.py gpurun_out/pmc_mf_2 gpurun_out/sq_mf_2 > /dev/null || exit 1
fi
if [ -n "${AB:-}" ]; then
  REPS=${REPS:-2} BENCH_ARGS="--steps 200 --warmup 5" bash tools/ab_env.sh $AB
fi
