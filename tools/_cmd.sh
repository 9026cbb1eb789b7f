set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r1b; mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1; rc=$?
tail -15 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --workload image --no-cpu-baseline > $O/bench_image.log 2>&1 && \
timeout -k 10 400 python bench.py --workload stream --steps 3 --warmup 1 > $O/bench_stream.log 2>&1
rc=$?; tail -2 $O/bench*.log; exit $rc
