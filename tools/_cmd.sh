timeout -k 10 600 python -m pytest tests/test_gpu_stream.py tests/test_gpu_codec.py -q -x > gpurun_out/zc_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/zc_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/zc_bench.log 2>&1
rc=$?; tail -1 gpurun_out/zc_bench.log; exit $rc
