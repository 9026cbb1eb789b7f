timeout -k 10 600 python -m pytest tests/test_gpu_codec.py -q -x -k "pyramid" > gpurun_out/pyr_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/pyr_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/bench_rows.py --rows image_linear_p0 --no-cpu > gpurun_out/il_rows.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/il_rows.log; exit $rc
