set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/trace; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -x -q --timeout 120 --timeout-method thread -k trace > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
KMP_TRACE=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/trace_demo.py > $O/log 2>&1; rc=$?
tail -2 $O/log; exit $rc
