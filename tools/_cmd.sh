timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/ch2_pytest.log 2>&1 && \
timeout -k 10 600 python tools/bench_rows.py --rows volume_chunks --no-cpu > gpurun_out/ch2_rows.log 2>&1
rc=$?; tail -2 gpurun_out/ch2_pytest.log; grep -v amdgpu gpurun_out/ch2_rows.log; exit $rc
