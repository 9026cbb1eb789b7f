set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s34; mkdir -p $O
timeout -k 10 400 python tools/bench_rows.py --no-cpu --rows volume_linear_p0,volume_linear_p1,volume_mean_p0,volume_mean_p1 > $O/rows.log 2>&1 || { tail -20 $O/rows.log; exit 1; }
grep '^{' $O/rows.log | cut -c1-200
