set -u
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_$i.json 2> $O/b20_$i.err || { tail -20 $O/b20_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b20_$i.json'));print('b20',d['value'],d['ms_per_step'],d['roofline']['frac'])"
done
for i in 1 2; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20q8_$i.json 2> $O/b20q8_$i.err || exit 1
  python -c "import json;d=json.load(open('$O/b20q8_$i.json'));print('b20q8',d['value'],d['ms_per_step'],d['roofline']['frac'])"
done
timeout -k 10 300 python bench.py --gpus 1 --steps 500 --warmup 5 > $O/b500.json 2> $O/b500.err || exit 1
python -c "import json;d=json.load(open('$O/b500.json'));print('b500',d['value'],d['ms_per_step'],d['roofline']['frac'])"
