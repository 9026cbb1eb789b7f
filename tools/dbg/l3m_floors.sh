set -o pipefail
O=gpurun_out/r4s13; mkdir -p $O
for v in "" e1 e2 e3 ""; do
  lib=kompressor_amd/libkompressor_hip${v:+_$v}.so
  KOMPRESSOR_HIP_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v$v -o run -- python3 tools/ktime.py volume 0 20 linearmx > $O/v$v.log 2>&1
  echo "== $lib"; python3 - $O/v$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'linear3m' in r['Name']: print(f"  {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:90]}")
PY
done
