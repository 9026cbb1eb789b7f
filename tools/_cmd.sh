timeout -k 10 600 python -m pytest tests/test_gpu_slabs.py -q -x > gpurun_out/slabs_pytest.log 2>&1
rc=$?; tail -30 gpurun_out/slabs_pytest.log; exit $rc
