#!/bin/bash
# NMS A/B: the NMS parity tests, then interleaved benches of the streaming certified NMS
# (uncapped grid, or SFMFEAT_NMS_STREAM_WG persistent workgroups) vs the tiled kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_nms.py -x -q --timeout 120 --timeout-method thread > $OUT/ab_pytest.log 2>&1 || { tail -30 $OUT/ab_pytest.log; exit 1; }
tail -2 $OUT/ab_pytest.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['stages_ms']['nms']['ms_per_step'])" $1; }
for i in 1 2; do
  for v in ${VARIANTS:-"stream:X=1" "wg1024:SFMFEAT_NMS_STREAM_WG=1024" "wg2048:SFMFEAT_NMS_STREAM_WG=2048" "wg4096:SFMFEAT_NMS_STREAM_WG=4096" "tile:SFMFEAT_NMS_TILE=1"}; do
    name=${v%%:*}; ev=${v#*:}
    env $ev timeout -k 10 300 python bench.py --steps 1000 --warmup 5 --cpu-sample 0 > $OUT/ab_${name}_$i.log 2>&1 || { tail -20 $OUT/ab_${name}_$i.log; exit 1; }
    show $OUT/ab_${name}_$i.log
  done
done
