#!/bin/bash
# Serial kernel durations (SFMFEAT_SERIAL=1, --inflight 1) of the certified NMS variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
export SFMFEAT_SERIAL=1
run() {  # run TAG ENV...
  local v=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ps_$v -o run -- python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-profile --inflight 1 > $OUT/ps_$v.log 2>&1 || exit 1
  f=$(find $OUT/ps_$v -name "*kernel_trace.csv" | head -1)
  python - "$f" $v <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
n = [r for r in rows if 'nms' in r['Kernel_Name'] and '1, 1' not in r['Kernel_Name']]
print(sys.argv[2], ' '.join('%.1f' % ((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3) for r in n[-12:]))
PY
}
run sh4 SFMFEAT_NMS_SH=4
run sh8 SFMFEAT_NMS_SH=8
run sh16 SFMFEAT_NMS_SH=16
run tile SFMFEAT_NMS_TILE=1
