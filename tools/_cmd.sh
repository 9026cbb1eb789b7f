set -o pipefail
mkdir -p gpurun_out/l3p
timeout -k 10 600 python -u -m pytest tests/test_gpu_linear.py -x -v --timeout 120 --timeout-method thread > gpurun_out/l3p/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/l3p/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/l3p/pytest.log | head -80; exit $rc; }
timeout -k 10 300 python tools/bench_rows.py --rows volume_linear_p1 --no-cpu > gpurun_out/l3p/rows1.log 2>&1
rc=$?; grep -h row gpurun_out/l3p/rows*.log; exit $rc
