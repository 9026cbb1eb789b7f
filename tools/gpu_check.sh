#!/bin/bash
# One gpurun call: GPU parity tests, smoke, bench, rocprof kernel stats.  Every GPU step has its
# own time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-check}
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-e2e --steps 20 > $OUT/prof.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log; cat $OUT/bench.log | tail -2
exit $rc
