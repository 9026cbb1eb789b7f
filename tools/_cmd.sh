set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s17; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_packing.py tests/test_gpu_container.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for lib in libkompressor_hip.so libkompressor_hip_prev.so libkompressor_hip.so libkompressor_hip_prev.so; do
  rm -rf $O/p
  KOMPRESSOR_HIP_LIB=$PWD/kompressor_amd/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/rice_time.py 4 20 > $O/run_$lib.log 2>&1
  f=$(find $O/p -name 'run_kernel_stats.csv' | head -1)
  echo "== $lib $(tail -1 $O/run_$lib.log)"
  python3 tools/kcsv.py $f rice_bundle_encode
done
timeout -k 10 300 python tools/host_rice.py > $O/host.log 2>&1 || { tail -30 $O/host.log; exit 1; }
grep "per call" $O/host.log
