set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/r4r1; mkdir -p $O
for v in "" _w4 "" _w4; do
  echo "== $v" >> $O/ab.log
  KOMPRESSOR_HIP_LIB=$PWD/kompressor_amd/libkompressor_hip$v.so timeout -k 10 200 python -u tools/bench_rows.py --rows rice --no-cpu --reps 10 2>&1 | grep '"rice' | grep device >> $O/ab.log || exit 1
done
cut -c1-150 $O/ab.log
