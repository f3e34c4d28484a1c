for a in ${ABLS:-0 8 9 10}; do
  SFMFEAT_MATCH_ABL=$a timeout -k 5 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abl$a -o run -- python tools/bench_match.py --iters 20 > gpurun_out/abl$a.log 2>&1 || exit 1
  grep -h "k_match_mfma" gpurun_out/abl$a/run_kernel_stats.csv | cut -d, -f2-4
done
