set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s30; mkdir -p $O
timeout -k 10 300 python tools/bench_rows.py --no-cpu --rows rice > $O/rows.log 2>&1 || { tail -20 $O/rows.log; exit 1; }
grep '^{' $O/rows.log | grep "device" | cut -c1-220
KMP_FUZZ_RICE_CASES=1500 KMP_FUZZ_SEED0=1000 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz_rice.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/fuzz_rice.log 2>&1 || { tail -20 $O/fuzz_rice.log; exit 1; }
tail -1 $O/fuzz_rice.log
KMP_FUZZ_CASES=3000 KMP_FUZZ_SEED0=30000 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_fuzz_primitives.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/fuzz.log 2>&1 || { tail -20 $O/fuzz.log; exit 1; }
tail -1 $O/fuzz.log
