set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pk; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_packing.py tests/test_gpu_codec.py -k "pack or wave2d_u8" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -80; exit $rc; }
for rep in 1 2; do for lib in tools/ab_base.so kompressor_amd/libkompressor_hip.so; do
  KOMPRESSOR_HIP_LIB=$PWD/$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$rep$(basename $lib) -o run -- python3 tools/bench_rows.py --rows packing --no-cpu > $O/rows_$rep$(basename $lib).log 2>&1 || exit 1
  grep -h '"row"' $O/rows_$rep$(basename $lib).log | cut -c1-150
  f=$(find $O/$rep$(basename $lib) -name 'run_kernel_stats.csv'); python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    n = r['Name']
    if 'kmp::pk' in n: print('$(basename $lib)', 'rep=$rep', round(float(r['AverageNs'])/1e3,2), n.split('(')[0][-40:])
"
done; done
