timeout -k 10 600 python -m pytest tests/test_gpu_codec.py -q -x -k categorical > gpurun_out/cat_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/cat_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/bench_rows.py --rows categorical --no-cpu > gpurun_out/cat_rows.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/cat_rows.log; exit $rc
