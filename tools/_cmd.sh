set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pkprof; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_packing.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -80; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/bench_rows.py --rows packing --no-cpu > $O/log 2>&1; rc=$?
grep -h row $O/log | cut -c1-200; exit $rc
