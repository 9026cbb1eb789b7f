#!/bin/bash
# Round-end evidence in one gpurun call: tools/gpu_round.sh (GPU parity suite, smoke, C3 / C2 / C5
# bench lines, rocprofv3 kernel stats, FETCH_SIZE / WRITE_SIZE passes), then the parity subset
# against the KMP_DEBUG=1 library and the N = 2 bench path rehearsed with gloo on one GPU.  Each GPU
# step has its own time limit; the chain stops at the first failure.
#   bash tools/gpu_final.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-final}
mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc"; return $rc; }
bash tools/gpu_round.sh ${1:-final} && \
step debug_parity 600 env KMP_DEBUG=1 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_linear.py tests/test_packing.py -m gpu -x -q --timeout 120 --timeout-method thread && \
step bench_n2_gloo 300 env KMP_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 5 --warmup 2 --no-e2e
rc=$?
tail -2 $O/debug_parity.log; tail -1 $O/bench_n2_gloo.log
exit $rc
