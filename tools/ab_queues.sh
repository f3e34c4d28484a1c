cd $GRAFT_REPO_ROOT
for q in ${QS:-4 8 16 4 8 16}; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --cpu-sample 0 --no-profile > gpurun_out/abq_$q.log 2>&1 || exit 1
  echo "q=$q $(tail -1 gpurun_out/abq_$q.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
