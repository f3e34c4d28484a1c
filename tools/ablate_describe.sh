#!/bin/bash
# Describe timing ablations (SFMFEAT_DQ_ABL, describe_q.hip): kernel trace per variant.
# (timing ablations: needs the diagnostic library, `make -C sfmfromscratch_amd/csrc ABLATIONS=1`)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for A in ${ABLS:-0 1 2 4 8 7 16 32 64 55 127}; do
  SFMFEAT_LIB=$PWD/sfmfromscratch_amd/lib_diag/libsfmfeat.so SFMFEAT_SERIAL=1 SFMFEAT_DQ_ABL=$A timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/dqabl_$A -o run -- \
    python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-profile --ablation-run > $OUT/dqabl_$A.log 2>&1 || exit 1
  python - "$A" <<'PY'
import csv, glob, sys
a = sys.argv[1]
p = glob.glob(f"gpurun_out/dqabl_{a}/**/*kernel_trace.csv", recursive=True)[0]
d = {}
for r in csv.DictReader(open(p)):
    n = r["Kernel_Name"]
    if "k_describe_q<" in n:
        k = n.split("(")[0].replace("void ", "").replace("sfm::dq::", "")
        d.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items()):
    print(f"ABL {a}: {k:32s} n={len(v):3d} mean={sum(v)/len(v):8.1f} us min={min(v):8.1f}")
PY
done
