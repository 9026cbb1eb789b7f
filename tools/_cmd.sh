set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lin; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -60; exit $rc; }
timeout -k 10 300 python tools/bench_rows.py --rows volume_linear_p0,volume_linear_p1 --no-cpu > $O/rows.log 2>&1; rc=$?
grep -h row $O/rows.log | cut -c1-160; exit $rc
