set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s40; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_packing.py tests/test_gpu_container.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/host_rice.py > $O/host.log 2>&1 || { tail -30 $O/host.log; exit 1; }
grep "per call" $O/host.log
timeout -k 10 300 python tools/bench_rows.py --no-cpu --rows rice > $O/rows.log 2>&1 || exit 1
grep -h '"rice:noise[0-9]*"' $O/rows.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['row'], d['pack_encoded_ms'], d['unpack_encoded_ms'], d['pack_device_us'], d['unpack_device_us'])"
