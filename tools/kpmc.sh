#!/bin/bash
# rocprofv3 HBM-traffic sweep (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md):
#   bash tools/kpmc.sh OUTDIR WORKLOAD "ENV=.." ...
set -o pipefail
export TMPDIR=/tmp
O=$1; WL=$2; shift 2
mkdir -p $O
i=0
for cfg in "$@"; do
  i=$((i+1))
  for ctr in FETCH_SIZE WRITE_SIZE; do
    ( for kv in $cfg; do export "$kv"; done
      timeout -k 10 120 rocprofv3 --pmc $ctr --output-format csv -d $O/c$i$ctr -o run -- python3 tools/ktime.py $WL 0 5 > $O/c$i$ctr.log 2>&1 ) || exit 1
  done
  echo "== [$cfg]"
  python3 - $O/c${i}FETCH_SIZE $O/c${i}WRITE_SIZE <<'PY'
import csv, sys, glob, collections
vals = collections.defaultdict(list)
for d in sys.argv[1:]:
    f = glob.glob(d + '/**/run_counter_collection.csv', recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if 'kmp' in r['Kernel_Name']:
            vals[(r['Kernel_Name'][:70], r['Counter_Name'])].append(float(r['Counter_Value']))
names = sorted({k[0] for k in vals})
for n in names:
    fe = sum(vals[(n, 'FETCH_SIZE')]) / max(1, len(vals[(n, 'FETCH_SIZE')]))
    wr = sum(vals[(n, 'WRITE_SIZE')]) / max(1, len(vals[(n, 'WRITE_SIZE')]))
    print(f"  fetch x2 {2*fe/1024:8.1f} MiB  write {wr/1024:8.1f} MiB  hbm {(2*fe+wr)/1024:8.1f} MiB  {n}")
PY
done
