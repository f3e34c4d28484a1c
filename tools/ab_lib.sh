#!/bin/bash
# Same-box A/B of two builds of libsfmfeat.so: the matcher sweep alone (tools/ab_kernel.sh) and
# the driver's bench command, interleaved A B A B.  A = ab_head/base (a saved build), B = the
# in-tree library.  usage: bash tools/ab_lib.sh [kernel-substring]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=$PWD/ab_head/base/libsfmfeat.so
B=$PWD/sfmfromscratch_amd/lib/libsfmfeat.so
K=${1:-k_match_mfma}
VAR=SFMFEAT_LIB VALS="$A $B $A $B" KERNEL=$K timeout -k 10 400 bash tools/ab_kernel.sh || exit 1
for v in A B A B; do
  lib=$A; [ $v = B ] && lib=$B
  SFMFEAT_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ablib_$v.json 2> gpurun_out/ablib_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ablib_$v.json'));print('$v', d['value'], d['ms_per_step'], d['library']['path'])"
done
