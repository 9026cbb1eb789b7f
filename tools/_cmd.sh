timeout -k 10 600 python -m pytest tests/test_gpu_linear.py tests/test_gpu_codec.py -q -x > gpurun_out/l3_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/l3_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/bench_rows.py --rows volume_linear_p0,volume_linear_p1 --no-cpu > gpurun_out/l3_rows.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/l3_rows.log; exit $rc
