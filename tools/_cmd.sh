set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mp; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_primitives.py tests/test_gpu_codec.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -80; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/bench_rows.py --rows volume_callback --no-cpu > $O/log 2>&1; rc=$?
grep -h '"row"' $O/log | cut -c1-170
f=$(find $O/p -name 'run_kernel_stats.csv'); python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'kmp' in r['Name']: print(round(float(r['AverageNs'])/1e3,2), r['Calls'], r['Name'][:70])
"; exit $rc
