set -o pipefail
mkdir -p gpurun_out/pk
timeout -k 10 600 python -u -m pytest tests/test_packing.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pk/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/pk/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/pk/pytest.log | head -80; exit $rc; }
timeout -k 10 300 python tools/bench_rows.py --rows packing --no-cpu > gpurun_out/pk/rows.log 2>&1
rc=$?; grep -h row gpurun_out/pk/rows.log; tail -3 gpurun_out/pk/rows.log; exit $rc
