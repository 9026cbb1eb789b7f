set -o pipefail
mkdir -p gpurun_out/w3p
timeout -k 10 300 python tools/sweep.py volume 2 '[{},{"KMP_W3P_PL":"1","KMP_W3P_WPE":"1"},{"KMP_W3P_PL":"2","KMP_W3P_WPE":"3"},{"KMP_W3P_PL":"1","KMP_W3P_WPE":"3"}]' > gpurun_out/w3p/sweep2b.log 2>&1 && \
timeout -k 10 300 python tools/bench_rows.py --rows volume_mean_p2 --no-cpu --reps 50 > gpurun_out/w3p/rows2.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/w3p/sweep2b.log gpurun_out/w3p/rows2.log; exit $rc
