timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/idx_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/idx_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/bench_rows.py --rows primitives,volume_callback,volume_linear_p1,categorical --no-cpu > gpurun_out/idx_rows.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/idx_rows.log; exit $rc
