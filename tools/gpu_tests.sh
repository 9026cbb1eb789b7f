#!/bin/bash
# The GPU test suite (or the files given) in one process, with its own time limit.
#   bash tools/gpu_tests.sh TAG [pytest args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-tests}; shift
mkdir -p $O
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
exit $rc
