timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/wide_pytest.log 2>&1; rc=$?
tail -8 gpurun_out/wide_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/bench_rows.py --rows volume_global,volume_mean_p0 --no-cpu > gpurun_out/wide_rows.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/wide_rows.log; exit $rc
