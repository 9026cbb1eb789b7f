timeout -k 10 600 python tools/bench_rows.py > gpurun_out/rows1.log 2>&1
rc=$?; cat gpurun_out/rows1.log | grep -v amdgpu.ids; exit $rc
