#!/bin/bash
# Quick GPU check in one gpurun call: the GPU parity suite, the bench lines (C3 / C2 / C5 with the
# CPU baselines), the parity subset against the KMP_DEBUG=1 library (device bounds checks), and
# the N = 2 bench path rehearsed with gloo on one GPU.  Each step has its own time limit; the
# chain stops at the first failure.   bash tools/gpu_quick.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-quick}
mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc"; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
step bench 400 python bench.py && \
step bench_image 300 python bench.py --workload image && \
step bench_stream 400 python bench.py --workload stream && \
step debug_parity 600 env KMP_DEBUG=1 python -u -m pytest tests/test_gpu_codec.py tests/test_packing.py -m gpu -x -q --timeout 120 --timeout-method thread && \
step bench_n2_gloo 300 env KMP_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 5 --warmup 2 --no-e2e
rc=$?
tail -3 $O/pytest_gpu.log; tail -1 $O/bench.log; tail -1 $O/bench_image.log; tail -1 $O/bench_stream.log; tail -2 $O/debug_parity.log; tail -1 $O/bench_n2_gloo.log
exit $rc
