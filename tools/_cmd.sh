set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab; rm -rf $O; mkdir -p $O
for rep in 1 2 3; do for v in 0 1; do
  KMP_W3_DEC_ORDER=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v${v}_$rep -o run -- python3 tools/ktime.py volume 0 30 > $O/v${v}_$rep.log 2>&1 || exit 1
  f=$(find $O/v${v}_$rep -name 'run_kernel_stats.csv'); python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'wave3d_plane' in r['Name']: print('order=$v rep=$rep', round(float(r['AverageNs'])/1e3,2), 'DEC' if 'true' in r['Name'] else 'ENC')
"
done; done
