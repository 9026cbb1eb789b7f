#!/bin/bash
# Alternating same-box A/B of an environment knob on the bench.py C3 line:
#   bash tools/ab_env.sh OUT VAR "v1 v2 ..." [reps] [bench args]
# prints "VAR=v value ms_encode ms_decode" per run
set -o pipefail
O=$1; VAR=$2; VALS=$3; REPS=${4:-2}; shift 4
mkdir -p $(dirname $O)
for r in $(seq $REPS); do
  for v in $VALS; do
    line=$(env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e "$@" 2>/dev/null | tail -1) || exit 1
    echo "$VAR=$v $(echo "$line" | python3 -c 'import sys, json; d = json.loads(sys.stdin.read()); print(d["value"], d["ms_encode"], d["ms_decode"])')" | tee -a $O
  done
done
