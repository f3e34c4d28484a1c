#!/bin/bash
# Fill-launch A/B: the GPU suite, then interleaved benches with the histogram / counter
# zeroing folded into k_down2x3 (default) vs two separate fill launches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/abf_pytest.log 2>&1 || { tail -30 $OUT/abf_pytest.log; exit 1; }
tail -2 $OUT/abf_pytest.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
for i in 1 2 3; do
  for v in "fold:X=1" "fill:SFMFEAT_FILL_LAUNCHES=1"; do
    name=${v%%:*}; ev=${v#*:}
    env $ev timeout -k 10 300 python bench.py --steps 1000 --warmup 5 --cpu-sample 0 > $OUT/abf_${name}_$i.log 2>&1 || { tail -20 $OUT/abf_${name}_$i.log; exit 1; }
    show $OUT/abf_${name}_$i.log
  done
done
