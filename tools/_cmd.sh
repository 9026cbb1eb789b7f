set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/reord; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -x -q --timeout 120 --timeout-method thread -k "golden or wide or metric" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 bench.py --no-cpu-baseline --no-e2e --steps 40 > $O/bench.log 2>&1; rc=$?
tail -1 $O/bench.log | cut -c1-400; exit $rc
