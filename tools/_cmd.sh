set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s22; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fuzz.py tests/test_gpu_graphs.py tests/test_gpu_rows.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python tools/bench_rows.py --no-cpu --rows volume_callback,volume_callback_f32,categorical > $O/rows.log 2>&1 || { tail -20 $O/rows.log; exit 1; }
grep '^{' $O/rows.log | grep -v "_cast\|_steps" | cut -c1-200
