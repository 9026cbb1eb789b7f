mkdir -p gpurun_out/r2s
bash tools/sq_counters.sh gpurun_out/r2s/sq "volume 1 3 linear" "KMP_L3R=1" > gpurun_out/r2s/sq.txt 2>&1 || exit 1
for z in 8 16 32; do echo "ZPER=$z" >> gpurun_out/r2s/zper.log; KMP_L3R_ZPER=$z timeout -k 10 200 python tools/bench_rows.py --rows volume_linear_p1 --no-cpu >> gpurun_out/r2s/zper.log 2>&1 || exit 1; done
grep -v "per dispatch" gpurun_out/r2s/sq.txt; grep -v amdgpu gpurun_out/r2s/zper.log | cut -c1-150
