#!/bin/bash
# SQ / LDS counters of Harris alone (tools/harris_alone.py: 32 planes per level, product kernel).
# Two --pmc passes, each under its own time limit; summaries via tools/sq_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r06_hpmc}
O=gpurun_out
LIB=${LIB:-}
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/${T}_p1 -o run -- python tools/harris_alone.py 5 $LIB > $O/${T}_p1.log 2>&1 || { echo "pass 1 rc=$?"; tail -5 $O/${T}_p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/${T}_p2 -o run -- python tools/harris_alone.py 5 $LIB > $O/${T}_p2.log 2>&1 || { echo "pass 2 rc=$?"; tail -5 $O/${T}_p2.log; exit 1; }
python tools/sq_summary.py $O/${T}_p1 $O/${T}_sq1 "$T pass 1" > /dev/null
python tools/sq_summary.py $O/${T}_p2 $O/${T}_sq2 "$T pass 2" > /dev/null
cat $O/${T}_sq1.txt
python - <<PY
import json
for p in ("$O/${T}_sq1.json", "$O/${T}_sq2.json"):
    d = json.load(open(p))
    for k, v in d.items():
        if "k_harris" in k:
            print(k[:60], v)
PY
