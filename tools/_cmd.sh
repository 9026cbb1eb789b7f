set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s32; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wave2d or image or golden" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
for lib in libkompressor_hip.so libkompressor_hip_prev.so; do
  rm -rf $O/p
  KOMPRESSOR_HIP_LIB=$PWD/kompressor_amd/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/ktime.py image 0 20 > $O/run.log 2>&1 || exit 1
  echo "== $lib $(python3 tools/kcsv.py $(find $O/p -name 'run_kernel_stats.csv' | head -1) wave2d | tr '\n' ' ' | cut -c1-200)"
done
done
