timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/p3_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/p3_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/bench_rows.py --rows volume_mean_p1,volume_mean_p2 --no-cpu > gpurun_out/p3_rows.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/p3_rows.log; exit $rc
