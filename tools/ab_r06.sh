#!/bin/bash
# Interleaved same-box A/B of the headline bench: base library (ab/base/libsfmfeat.so, or
# $BASE) vs the tree's library, N rounds, plus optional extra variants given as
# "name|ENV=VAL ...|bench args" in $VARIANTS (';'-separated).  Each run has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r06_ab}
N=${N:-3}
ARGS=${ARGS:---steps 200 --cpu-sample 0 --no-profile}
BASE=${BASE:-ab/base/libsfmfeat.so}
run() {  # run NAME ENV... -- ARGS
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py $ARGS ${EXTRA:-} > $O/${T}_$name.out 2> $O/${T}_$name.err || { echo "$name failed"; tail -5 $O/${T}_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${T}_$name.out'));r=d['roofline'] or {};print('$name', d['value'], d['ms_per_step'], r.get('frac'), (r.get('launch_sum') or {}).get('frac'))"
}
for i in $(seq 1 $N); do
  run base_$i SFMFEAT_LIB=$BASE
  run new_$i X=1
  IFS=';' read -ra VS <<< "${VARIANTS:-}"
  for v in "${VS[@]}"; do
    IFS='|' read -r vn venv vargs <<< "$v"
    EXTRA="$vargs" run ${vn}_$i $venv X=1
  done
done
