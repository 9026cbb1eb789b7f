#!/bin/bash
# Round-3 measurement batch in one gpurun call: secondary rows (callback u16 / f32 maps,
# categorical, Rice), the store-policy pipeline rows, and SQ counters of the Rice bundle and
# categorical kernels.  Each GPU step has its own time limit; the chain stops at the first failure.
#   bash tools/r3_probe.sh TAG [rows]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-probe}
ROWS=${2:-volume_callback,volume_callback_f32,categorical,rice}
mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc"; return $rc; }
step rows 600 python tools/bench_rows.py --no-cpu --rows $ROWS && \
step pipeline 300 python tools/pipeline_rows.py && \
step sq_rice 300 bash tools/sq_counters.sh $O/sq_rice "rice 4 10" && \
step sq_cat 300 bash tools/sq_counters.sh $O/sq_cat "categorical 0 5"
rc=$?
cat $O/rows.log | grep '^{'; grep '^{' $O/pipeline.log; cat $O/sq_rice.log $O/sq_cat.log
exit $rc
