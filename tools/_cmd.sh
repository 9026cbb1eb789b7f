set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s35; mkdir -p $O
KMP_FUZZ_RICE_CASES=4000 KMP_FUZZ_SEED0=3000 timeout -k 10 1000 python -u -m pytest tests/test_gpu_fuzz_rice.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/fuzz_rice.log 2>&1 || { tail -20 $O/fuzz_rice.log; exit 1; }
tail -1 $O/fuzz_rice.log
KMP_FUZZ_CASES=10000 KMP_FUZZ_SEED0=40000 timeout -k 10 1000 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_fuzz_primitives.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/fuzz.log 2>&1 || { tail -20 $O/fuzz.log; exit 1; }
tail -1 $O/fuzz.log
