#!/bin/bash
# NMS A/B: GPU suite, then bench with the streaming certified NMS vs the tiled kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/ab_pytest.log 2>&1 || { tail -30 $OUT/ab_pytest.log; exit 1; }
tail -2 $OUT/ab_pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 500 --warmup 3 --cpu-sample 0 > $OUT/ab_stream_$i.log 2>&1 || { tail -20 $OUT/ab_stream_$i.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['stages_ms']['nms'])" $OUT/ab_stream_$i.log
  SFMFEAT_NMS_TILE=1 timeout -k 10 300 python bench.py --steps 500 --warmup 3 --cpu-sample 0 > $OUT/ab_tile_$i.log 2>&1 || { tail -20 $OUT/ab_tile_$i.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['stages_ms']['nms'])" $OUT/ab_tile_$i.log
done
