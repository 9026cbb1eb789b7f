set -o pipefail
O=gpurun_out/rows; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_primitives.py tests/test_gpu_codec.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -80; exit $rc; }
timeout -k 10 300 python tools/bench_rows.py --rows primitives --no-cpu > $O/rows.log 2>&1
rc=$?; grep -h row $O/rows.log | cut -c1-150; exit $rc
