#!/bin/bash
# rocprofv3 kernel-time sweep: one profiled process per configuration (env assignments as args).
#   bash tools/kprof.sh OUTDIR WORKLOAD "ENV=.. ENV=.." "ENV=.." ...
set -o pipefail
export TMPDIR=/tmp
O=$1; WL=$2; shift 2
mkdir -p $O
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg KMP_TAG="$cfg" true
  ( for kv in $cfg; do export "$kv"; done
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c$i -o run -- python3 tools/ktime.py $WL 0 20 > $O/c$i.log 2>&1 ) || exit 1
  f=$(find $O/c$i -name "run_kernel_stats.csv" | head -1)
  echo "== [$cfg]"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name']
    if 'kmp' in n:
        print(f"  {float(r['AverageNs'])/1e3:8.1f} us  x{r['Calls']:>3}  {n[:90]}")
PY
done
