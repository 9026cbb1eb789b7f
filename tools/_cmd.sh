set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/chk; rm -rf $O; mkdir -p $O
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/chunks_probe.py 5 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
tail -1 $O/run.log
f=$(find $O/p -name 'run_kernel_stats.csv'); python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    print(r['Calls'], round(float(r['AverageNs'])/1e3,2), r['Name'][:110])
"
f=$(find $O/p -name 'run_kernel_trace.csv'); python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in rows[-12:]:
    print(round((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3,2), r['Grid_Size_X'] if 'Grid_Size_X' in r else r.get('Grid_Size',''), r['Kernel_Name'][:80])
"
