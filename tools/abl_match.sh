#!/bin/bash
# Matcher sweep timing ablations (SFMFEAT_MATCH_ABL, match_mfma.hip; results wrong by design):
# the diagnostic library (make -C sfmfromscratch_amd/csrc ABLATIONS=1), tools/bench_match.py under
# a rocprofv3 kernel trace per variant; prints k_match_mfma's mean / min duration per variant.
#   0 full, 1 no epilogue, 2 no MFMAs, 4 no admission masks / appends, 6 = 2 + 4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in ${ABLS:-0 1 2 4 6}; do
  SFMFEAT_LIB=$PWD/sfmfromscratch_amd/lib_diag/libsfmfeat.so SFMFEAT_MATCH_ABL=$a timeout -k 5 120 \
    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mabl$a -o run -- \
    python tools/bench_match.py --iters 20 ${MATCH_ARGS:-} > gpurun_out/mabl$a.log 2>&1 || exit 1
  python - "$a" <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(f"gpurun_out/mabl{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_match_mfma" in r["Kernel_Name"]:
            rows.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
rows = rows[1:] or rows
print(f"MATCH_ABL={sys.argv[1]}: k_match_mfma {len(rows)} launches, mean {sum(rows) / max(len(rows), 1):.1f} us, min {min(rows):.1f} us")
PY
done
