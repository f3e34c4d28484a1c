#!/bin/bash
# Generic gpurun session: each argument is "name|seconds|command"; the steps run in order,
# each under its own time limit, and the first failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; to=${rest%%|*}; cmd=${rest#*|}
  echo "[$(date +%T)] $name: $cmd" >> $OUT/status.txt
  timeout -k 10 "$to" bash -c "$cmd" > $OUT/$name.log 2>&1; rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $OUT/status.txt
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; tail -30 $OUT/$name.log; exit $rc; fi
  echo "== $name ok"; tail -${TAILN:-3} $OUT/$name.log
done
