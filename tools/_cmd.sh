set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s37; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread -k categorical > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for lib in libkompressor_hip.so libkompressor_hip_prev.so; do
  KOMPRESSOR_HIP_LIB=$PWD/kompressor_amd/$lib timeout -k 10 300 python tools/bench_rows.py --no-cpu --rows categorical > $O/rows_$lib.log 2>&1 || exit 1
  echo "== $lib $(grep '^{' $O/rows_$lib.log | python3 -c "import sys,json; print(' '.join(json.loads(l)['row'].split(':')[1]+'='+str(json.loads(l)['us']) for l in sys.stdin))")"
done
done
