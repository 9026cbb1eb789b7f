#!/bin/bash
# Rice bundle iteration in one gpurun call: container parity tests, the rice rows, SQ counters of
# the bundle kernels.  Each GPU step has its own time limit; the chain stops at the first failure.
#   bash tools/r3_rice.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-rice}
mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc"; return $rc; }
step tests 300 python -u -m pytest tests/test_packing.py tests/test_gpu_container.py -m gpu -x -q --timeout 120 --timeout-method thread && \
step rows 300 python tools/bench_rows.py --no-cpu --rows rice && \
step sq_rice 300 bash tools/sq_counters.sh $O/sq_rice "rice 4 10"
rc=$?
tail -3 $O/tests.log; grep '^{' $O/rows.log | cut -c1-400; cat $O/sq_rice.log
exit $rc
