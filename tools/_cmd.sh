set -o pipefail
mkdir -p gpurun_out/cb
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_primitives.py -x -q --timeout 120 --timeout-method thread > gpurun_out/cb/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/cb/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/cb/pytest.log | head -80; exit $rc; }
timeout -k 10 300 python tools/bench_rows.py --rows volume_callback --no-cpu > gpurun_out/cb/rows.log 2>&1
rc=$?; grep -h row gpurun_out/cb/rows.log; exit $rc
