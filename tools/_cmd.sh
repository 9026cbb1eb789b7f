set -o pipefail
O=gpurun_out/capi; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_capi.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest.log | head -50; exit $rc; }
timeout -k 10 60 ./tools/capi_example 512 | tee $O/capi.log
