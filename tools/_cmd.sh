set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s41; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fuzz.py tests/test_gpu_graphs.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lib in libkompressor_hip.so libkompressor_hip_prev.so libkompressor_hip.so libkompressor_hip_prev.so; do
  rm -rf $O/p
  KOMPRESSOR_HIP_LIB=$PWD/kompressor_amd/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/callback_split.py 10 u16 > $O/kt.log 2>&1 || exit 1
  echo "== $lib $(python3 tools/kcsv.py $(find $O/p -name 'run_kernel_stats.csv' | head -1) 'true, 3' | cut -c1-14)"
done
for lib in libkompressor_hip.so libkompressor_hip_prev.so; do
  KOMPRESSOR_HIP_LIB=$PWD/kompressor_amd/$lib timeout -k 10 300 python tools/bench_rows.py --no-cpu --rows volume_callback > $O/rows_$lib.log 2>&1 || exit 1
  echo "== $lib $(grep '^{' $O/rows_$lib.log | grep -v _128 | python3 -c "import sys,json; print(' '.join(json.loads(l)['row'].split(':')[1]+'='+str(json.loads(l)['us'])+'/'+str(json.loads(l)['GBps']) for l in sys.stdin))")"
done
