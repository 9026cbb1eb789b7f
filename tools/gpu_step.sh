#!/bin/bash
# One GPU call of named steps, each under its own time limit, chained so the first failure ends it.
#   bash tools/gpu_step.sh TAG 'name:seconds:command' ['name:seconds:command' ...]
# Logs go to gpurun_out/TAG/<name>.log; the tail of each is printed at the end.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
rc=0
names=()
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  names+=("$name")
  timeout -k 10 "$secs" bash -c "$cmd" > $O/$name.log 2>&1
  rc=$?
  echo "[$name] rc=$rc"
  [ $rc -ne 0 ] && break
done
for n in "${names[@]}"; do echo "== $n"; tail -4 $O/$n.log; done
exit $rc
