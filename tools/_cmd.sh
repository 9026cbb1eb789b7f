set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s38; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_packing.py tests/test_gpu_container.py tests/test_gpu_fuzz_rice.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lib in libkompressor_hip.so libkompressor_hip_prev.so libkompressor_hip.so libkompressor_hip_prev.so; do
  rm -rf $O/p
  KOMPRESSOR_HIP_LIB=$PWD/kompressor_amd/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/rice_time.py 4 20 > $O/run_$lib.log 2>&1 || exit 1
  echo "== $lib $(tail -1 $O/run_$lib.log) $(python3 tools/kcsv.py $(find $O/p -name 'run_kernel_stats.csv' | head -1) rice_bundle_encode | cut -c1-20)"
done
timeout -k 10 300 python tools/bench_rows.py --no-cpu --rows rice > $O/rows.log 2>&1 || exit 1
grep -h '"rice:noise[0-9]*"' $O/rows.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['row'], d['pack_encoded_ms'], d['unpack_encoded_ms'], d['pack_device_us'], d['unpack_device_us'])"
grep compress_device $O/rows.log | cut -c1-200
