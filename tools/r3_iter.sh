#!/bin/bash
# Iteration batch in one gpurun call: the named GPU test files, the named bench rows, optional SQ
# counters of a ktime workload.  Each GPU step has its own time limit; the chain stops at the
# first failure.   bash tools/r3_iter.sh TAG "tests/a.py tests/b.py" "rows" ["ktime args"]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-iter}; TESTS=$2; ROWS=$3; SQ=$4
mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc"; return $rc; }
rc=0
if [ -n "$TESTS" ]; then step tests 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread || rc=1; fi
if [ $rc = 0 ] && [ -n "$ROWS" ]; then step rows 600 python tools/bench_rows.py --no-cpu --rows $ROWS || rc=1; fi
if [ $rc = 0 ] && [ -n "$SQ" ]; then step sq 300 bash tools/sq_counters.sh $O/sq "$SQ" || rc=1; fi
[ -f $O/tests.log ] && tail -3 $O/tests.log
[ -f $O/rows.log ] && grep '^{' $O/rows.log | cut -c1-420
[ -f $O/sq.log ] && cat $O/sq.log
exit $rc
