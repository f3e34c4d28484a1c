#!/bin/bash
# k_select timing ablations (SFMFEAT_SELECT_ABL, select.hip; results wrong by design): kernel
# (timing ablations: needs the diagnostic library, `make -C sfmfromscratch_amd/csrc ABLATIONS=1`)
# trace of a serial bench run per variant, mean / min duration per launch shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for A in ${ABLS:-0 1 2 3}; do
  SFMFEAT_LIB=$PWD/sfmfromscratch_amd/lib_diag/libsfmfeat.so SFMFEAT_SERIAL=1 SFMFEAT_SELECT_MERGE=0 SFMFEAT_SELECT_ABL=$A timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/selabl_$A -o run -- \
    python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-profile --ablation-run ${BENCH_ARGS:-} > gpurun_out/selabl_$A.log 2>&1 || exit 1
  python - "$A" "${LEVELS:-4}" <<'PY'
import csv, glob, sys
a = sys.argv[1]
p = glob.glob(f"gpurun_out/selabl_{a}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(p)))
sel = [(e - s) / 1e3 for s, e, n in rows if "k_select" in n]
# serial, unmerged: the launches of one extraction are the levels in order
L = int(sys.argv[2]) if len(sys.argv) > 2 else 4
for l in range(L):
    v = sel[l::L]
    print(f"ABL {a}: k_select level {l} n={len(v):3d} mean={sum(v)/len(v):8.1f} us min={min(v):8.1f}")
PY
done
