set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s26; mkdir -p $O
for lib in libkompressor_hip.so libkompressor_hip_prev.so libkompressor_hip.so libkompressor_hip_prev.so; do
  for w in u16 f32; do
  rm -rf $O/p
  KOMPRESSOR_HIP_LIB=$PWD/kompressor_amd/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/callback_split.py 10 $w > $O/kt.log 2>&1
  echo "== $lib $w"
  python3 tools/kcsv.py $(find $O/p -name 'run_kernel_stats.csv' | head -1) rows_code
  done
done
