#!/bin/bash
# Round evidence in one gpurun call: GPU parity tests, smoke, benches, rocprofv3 kernel stats and
# HBM-traffic PMC passes (FETCH_SIZE / WRITE_SIZE in separate passes).  Each GPU step has its own
# time limit; the chain stops at the first failure.
#   bash tools/gpu_round.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-round}
mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc"; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread && \
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" && \
step bench 400 python bench.py && \
step bench_image 300 python bench.py --workload image && \
step bench_stream 400 python bench.py --workload stream && \
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --no-e2e && \
step prof_image 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_image -o run -- python3 bench.py --workload image --no-cpu-baseline --no-e2e && \
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 && \
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 && \
step pmc_fetch_image 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_image -o run -- python3 bench.py --workload image --no-cpu-baseline --no-e2e --steps 3 --warmup 1 && \
step pmc_write_image 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_image -o run -- python3 bench.py --workload image --no-cpu-baseline --no-e2e --steps 3 --warmup 1
rc=$?
tail -2 $O/pytest_gpu.log; tail -1 $O/bench.log; tail -1 $O/bench_image.log; tail -1 $O/bench_stream.log
exit $rc
