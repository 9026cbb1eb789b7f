#!/bin/bash
# rocprofv3 kernel averages of tools/ktime.py (encode / decode alternating) for one workload and
# padding under several environment settings, one profiled process each:
#   bash tools/kprof_p.sh OUTDIR WORKLOAD PADDING "ENV=.. ENV=.." "ENV=.." ...
# WORKLOAD may carry the predictor kind: volume:linear
set -o pipefail
export TMPDIR=/tmp
O=$1; WL=${2%%:*}; KIND=; [[ $2 == *:* ]] && KIND=${2#*:}; PAD=$3; shift 3
mkdir -p $O
i=0
for cfg in "$@"; do
  i=$((i+1))
  ( for kv in $cfg; do export "$kv"; done
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c$i -o run -- python3 tools/ktime.py $WL $PAD 20 $KIND > $O/c$i.log 2>&1 ) || exit 1
  f=$(find $O/c$i -name "run_kernel_stats.csv" | head -1)
  echo "== [$WL p=$PAD $cfg]"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'kmp' in r['Name']:
        print(f"  {float(r['AverageNs'])/1e3:8.1f} us  x{r['Calls']:>3}  {r['Name'][:100]}")
PY
done
