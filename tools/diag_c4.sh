rm -f gpurun_out/c4b.log
echo "== c4 two-stream, CU-exclusive matcher" >> gpurun_out/c4b.log; timeout -k 10 200 python tools/check_c4b.py 256 two match >> gpurun_out/c4b.log 2>&1 || exit 1
