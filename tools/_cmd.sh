set -o pipefail
O=gpurun_out/rowsall; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u tools/bench_rows.py > $O/rows.log 2>&1; rc=$?
grep -h '"row"' $O/rows.log | cut -c1-170; exit $rc
