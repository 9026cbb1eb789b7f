set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s23; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz_rice.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -15 $O/tests.log
exit $rc
