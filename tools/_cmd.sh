set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s10; mkdir -p $O
timeout -k 10 300 python tools/bench_rows.py --no-cpu --rows rice > $O/rows.log 2>&1 || exit 1
grep -h '"rice:noise[0-9]*"' $O/rows.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['row'], d['pack_encoded_ms'], d['unpack_encoded_ms'], d['pack_device_us'], d['unpack_device_us'])"
timeout -k 10 300 bash tools/sq_counters.sh $O/sq "rice 4 10" > $O/sq.log 2>&1 || exit 1
cat $O/sq.log
