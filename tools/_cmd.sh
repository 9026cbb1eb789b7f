set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s54; mkdir -p $O
for lib in libkompressor_hip.so libkompressor_hip_pf8.so libkompressor_hip.so libkompressor_hip_pf8.so; do
  KOMPRESSOR_HIP_LIB=$PWD/kompressor_amd/$lib timeout -k 10 300 python tools/bench_rows.py --no-cpu --rows categorical > $O/rows_$lib.log 2>&1 || exit 1
  echo "== $lib $(grep '^{' $O/rows_$lib.log | python3 -c "import sys,json; print(' '.join(json.loads(l)['row'].split(':')[1]+'='+str(json.loads(l)['us']) for l in sys.stdin))")"
done
